// gfd_common.h -- shared device helpers for the gfx950 GATConv kernels.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "gfd.h"

namespace gfd {

constexpr int kWave = 64;
constexpr int kHeads = 8;      // the reference hard-codes heads=8 (gat.py:39,45,51)
constexpr int kChannels = 64;  // hidden_channels=64 (config.py:32)
constexpr float kSoftmaxEps = 1e-16f;  // PyG utils.softmax denominator epsilon
// Messages (self loop included) of the largest "light" destination of the tile
// stage: every row prefetched one tile ahead (gfd_stream.hip); the plan's class
// split (k_slot_desc) uses the same bound.  6 measured against 4 and 5
// (scripts/gpu_ab.sh, -DGFD_LIGHT_MAX=n variants): C5 105.0 -> 101.2 ms, C4
// unchanged within noise.
#ifndef GFD_LIGHT_MAX
#define GFD_LIGHT_MAX 6
#endif
constexpr int kLightMax = GFD_LIGHT_MAX;
// ... for bf16 rows: one message more.  Their light instance holds 7 rows a
// slot spill-free (fp32 rows spill at 7), and the 7-message rows leave the
// general tiles: C5 general + light -0.5 ms (profiles/r6s_light_bound_ab.txt).
// The plan's class_split[3] is this bound's general / light boundary.
#ifndef GFD_LIGHT_MAX_BF16
#define GFD_LIGHT_MAX_BF16 7
#endif
constexpr int kLightMaxBf16 = GFD_LIGHT_MAX_BF16;
static_assert(kLightMax <= 7 && kLightMaxBf16 <= 7, "light slots: at most 7 messages");
// Messages of the largest destination of the "short light" sub-class: the
// light tiles whose slots all have at most this many messages run a kernel
// instance that prefetches only that many rows per slot, and spends the
// registers so freed on a deeper A-fragment read-ahead (gfd_stream.hip).  The
// plan's third class boundary (k_slot_desc) uses the same bound.
#ifndef GFD_LIGHT_LO
#define GFD_LIGHT_LO 3
#endif
constexpr int kLightLo = GFD_LIGHT_LO;

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define GFD_HIP_CHECK(expr)                          \
  do {                                               \
    hipError_t _e = (expr);                          \
    if (_e != hipSuccess) return GFD_ERR_HIP;        \
  } while (0)

#define GFD_LAUNCH_CHECK()                           \
  do {                                               \
    if (hipGetLastError() != hipSuccess) return GFD_ERR_HIP; \
  } while (0)

__host__ __device__ inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

// Bump allocator over a caller-provided workspace.
struct Carve {
  char* base;
  size_t cap;
  size_t off = 0;
  bool ok = true;
  Carve(void* b, size_t c) : base(static_cast<char*>(b)), cap(c) {}
  template <typename T>
  T* take(size_t count) {
    size_t o = align_up(off, 256);
    size_t need = o + count * sizeof(T);
    if (base == nullptr || need > cap) { ok = false; off = need; return nullptr; }
    off = need;
    return reinterpret_cast<T*>(base + o);
  }
};

// Same sizes without a buffer (for *_workspace_size).
struct Sizer {
  size_t off = 0;
  template <typename T>
  void take(size_t count) { off = align_up(off, 256) + count * sizeof(T); }
};

__device__ __forceinline__ float leaky(float v, float slope) { return v > 0.f ? v : v * slope; }
// the same for 0 <= slope <= 1 (bit-identical, +-0 included): one multiply and one max
__device__ __forceinline__ float leaky01(float v, float slope) { return fmaxf(v, v * slope); }

// Round-to-nearest-even fp32 -> bf16 bits (inputs are finite here).
__device__ __forceinline__ uint16_t bf16_bits(float f) {
  uint32_t u = __float_as_uint(f);
  u += 0x7FFFu + ((u >> 16) & 1u);
  return static_cast<uint16_t>(u >> 16);
}
__device__ __forceinline__ float bf16_to_f32(uint16_t b) { return __uint_as_float(uint32_t(b) << 16); }

// Split 8 fp32 into hi = bf16(v), lo = bf16(v - hi): hi+lo carries ~16 mantissa bits.
__device__ __forceinline__ void split8(const float* v, bf16x8& hi, bf16x8& lo) {
  union { bf16x8 v; uint16_t u[8]; } h, l;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    uint16_t hb = bf16_bits(v[j]);
    h.u[j] = hb;
    l.u[j] = bf16_bits(v[j] - bf16_to_f32(hb));
  }
  hi = h.v;
  lo = l.v;
}

// Counter-based dropout mask (splitmix64 finaliser): keep iff u >= p.
__device__ __forceinline__ bool dropout_keep(uint64_t seed, uint32_t pos, uint32_t head, float p) {
  uint64_t z = seed ^ ((uint64_t(pos) << 3 | head) * 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  float u = float(uint32_t(z >> 40)) * (1.0f / 16777216.0f);
  return u >= p;
}

__device__ __forceinline__ int wave_uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

// max of non-negative floats into *dst (their bit patterns order like the
// values).  Skips the atomic when *dst already holds at least v: thousands of
// same-address atomics otherwise serialise in L2 (one per wave of a large grid).
__device__ __forceinline__ void atomic_max_nonneg(float* dst, float v) {
  unsigned int* p = reinterpret_cast<unsigned int*>(dst);
  const unsigned int bits = __float_as_uint(v);
  if (bits > __atomic_load_n(p, __ATOMIC_RELAXED)) atomicMax(p, bits);
}

}  // namespace gfd
