// gfd_gat_fwd.hip -- GATConv forward for gfx950 (PyG GATConv.forward, concat=False;
// called at /root/reference/src/models/gat.py:80 and tgn.py:94).
//
// Dataflow (aggregate-then-project; SURVEY.md §7 "hard parts"):
//   k_wmax/k_pack  W [H*C,F], att -> folded logit vectors U/V [2H][Fu] and the
//                  fp16 hi/lo MFMA B-fragments of Wcat[(h,f)][c] = W[h*C+c][f]/H
//                  scaled by a power of two 2^kw (max |W| -> 2^14)
//   k_logits       st[n] = (x_n.U_h, x_n.V_h) on fp32 MFMA (exact fp32 chains)
//   k_fused        per 16-destination tile (rows taken in descending-degree order):
//     phase A      one destination per wave: online softmax over its CSR segment
//                  (max of leaky(s_j + t_i), p = exp(e - max)), z_ih += p x_j with
//                  the x row gathered once for all 8 heads, z /= sum p + 1e-16
//     phase B      out = Z . Wcat + bias on f16 MFMA 16x16x32, two head-halves
//                  through a 43 KB LDS tile; 3-term split hi.hi + (hi.lo + lo.hi)/2^11
//                  on power-of-two-scaled rows: ~2^-21 relative, fp32-faithful
//   k_hub_*        destinations with > threshold messages: chunk partials, per-hub
//                  (max, sum), merged z rows read by the tile kernel
#include <stdlib.h>

#include <type_traits>

#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int H = kHeads;
constexpr int C = kChannels;
constexpr int kTile = 16;       // destinations per fused block (MFMA M)
constexpr int kFusedWaves = 16; // one destination per wave
constexpr float kScaleTarget = 16384.f;  // 2^14: scaled |values| stay inside fp16
constexpr float kLoScale = 2048.f;        // 2^11: lo parts re-normalised into fp16

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));

struct PackLayout {
  int F, Fp, Fu, KP, KS, KH;
  size_t hdr_off, uv_off, whi_off, wlo_off, wsh_off, wsl_off, bytes;
};

inline PackLayout pack_layout(int F) {
  PackLayout L;
  L.F = F;
  L.Fp = (F + 7) / 8 * 8;   // K per head; 4*Fp (a head-half) is a multiple of 32
  L.Fu = (F + 15) / 16 * 16; // logit-vector row stride (vector loads never cross rows)
  L.KP = H * L.Fp;
  L.KS = L.KP / 32;          // MFMA k-steps
  L.KH = L.KS / 2;           // k-steps per head-half
  size_t o = 0;
  L.hdr_off = o; o = align_up(o + 64, 256);
  L.uv_off = o; o = align_up(o + sizeof(float) * 2 * H * L.Fu, 256);
  L.whi_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.wlo_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  // feature-major fragments for k_stream: K position p = 8 f + h, unscaled lo
  L.wsh_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.wsl_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.bytes = o;
  return L;
}

struct PackHeader {  // device-side, written by k_wmax
  float w_unscale;   // 2^-kw
  float w_scale;     // 2^kw
};

// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(1024) k_wmax(const float* __restrict__ W, int n,
                                               PackHeader* __restrict__ hdr) {
  // one block; 16-B loads when W is aligned, four independent chains per thread
  __shared__ float red[1024];
  const int t = threadIdx.x;
  float m0 = 0.f, m1 = 0.f, m2 = 0.f, m3 = 0.f;
  int i0 = 0;
  if ((reinterpret_cast<uintptr_t>(W) & 15) == 0) {
    const f32x4* W4 = reinterpret_cast<const f32x4*>(W);
    const int n4 = n >> 2;
    for (int i = t; i < n4; i += 1024) {
      const f32x4 w = W4[i];
      m0 = fmaxf(m0, fabsf(w.x));
      m1 = fmaxf(m1, fabsf(w.y));
      m2 = fmaxf(m2, fabsf(w.z));
      m3 = fmaxf(m3, fabsf(w.w));
    }
    i0 = n4 << 2;
  }
  for (int i = i0 + t; i < n; i += 1024) m0 = fmaxf(m0, fabsf(W[i]));
  red[t] = fmaxf(fmaxf(m0, m1), fmaxf(m2, m3));
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s) red[t] = fmaxf(red[t], red[t + s]);
    __syncthreads();
  }
  if (t == 0) {
    const float wm = red[0] * (1.0f / H);  // the packed values are W / H
    int ex = 0;
    if (wm > 0.f) frexpf(wm, &ex);         // wm < 2^ex
    int kw = 14 - ex;
    kw = kw > 100 ? 100 : (kw < -100 ? -100 : kw);
    hdr->w_scale = ldexpf(1.0f, kw);
    hdr->w_unscale = ldexpf(1.0f, -kw);
  }
}

__global__ void k_pack_uv(const float* __restrict__ W, const float* __restrict__ as,
                          const float* __restrict__ ad, int F, int Fu, float* __restrict__ uv) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2 * H * Fu) return;
  int q = idx / Fu, f = idx % Fu;
  int h = q % H;
  const float* a = (q < H ? as : ad) + h * C;
  float acc = 0.f;
  if (f < F) {
    for (int c = 0; c < C; ++c) acc = fmaf(a[c], W[size_t(h * C + c) * F + f], acc);
  }
  uv[idx] = acc;
}

__global__ void k_pack_frag(const float* __restrict__ W, int F, int Fp, int KS,
                            const PackHeader* __restrict__ hdr, uint4* __restrict__ whi,
                            uint4* __restrict__ wlo) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (s, ct, lane)
  if (idx >= KS * 4 * 64) return;
  int lane = idx & 63, ct = (idx >> 6) & 3, s = idx >> 8;
  int n = ct * 16 + (lane & 15);
  const float sc = hdr->w_scale * (1.0f / H);
  union { uint4 v; _Float16 h[8]; } hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int k = 32 * s + 8 * (lane >> 4) + j;
    int h = k / Fp, f = k % Fp;
    float v = (f < F) ? W[size_t(h * C + n) * F + f] * sc : 0.f;
    _Float16 hv = (_Float16)v;
    hi.h[j] = hv;
    lo.h[j] = (_Float16)((v - (float)hv) * kLoScale);
  }
  whi[idx] = hi.v;
  wlo[idx] = lo.v;
}

// Feature-major fragments for k_stream: K position p = 8 f + h (one 16-B Z store
// per feature holds all 8 heads), lo = v - hi unscaled (|lo| <= 2^3 for the
// 2^14-scaled W; fp16 subnormals there cost < 2^-38 of the largest weight).
__global__ void k_pack_frag_s(const float* __restrict__ W, int F, int KS,
                              const PackHeader* __restrict__ hdr, uint4* __restrict__ wsh,
                              uint4* __restrict__ wsl) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (s, ct, lane)
  if (idx >= KS * 4 * 64) return;
  int lane = idx & 63, ct = (idx >> 6) & 3, s = idx >> 8;
  int n = ct * 16 + (lane & 15);
  int f = 4 * s + (lane >> 4);
  const float sc = hdr->w_scale * (1.0f / H);
  union { uint4 v; _Float16 h[8]; } hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float v = (f < F) ? W[size_t(j * C + n) * F + f] * sc : 0.f;
    _Float16 hv = (_Float16)v;
    hi.h[j] = hv;
    lo.h[j] = (_Float16)(v - (float)hv);
  }
  wsh[idx] = hi.v;
  wsl[idx] = lo.v;
}

// ---------------------------------------------------------------------------
// st[r][q] = sum_f x[r][f] * uv[q][f] (q < 2H) on v_mfma_f32_16x16x4_f32.  A
// wave computes 16 rows x 16 logits.  Lane group g = l >> 4 reads VEC
// consecutive features k0 + VEC*g .. of its row l & 15 (one vector load), and
// MFMA step t pairs them with uv[l & 15][k0 + VEC*g + t]: the k order inside a
// 4*VEC block is permuted identically on both operands, so the sum is exact
// fp32 FMA chains over all F features.
template <int VEC>
__global__ void __launch_bounds__(256) k_logits(const float* __restrict__ x, int64_t rows, int F,
                                                int64_t ldx, const float* __restrict__ uv, int Fu,
                                                float* __restrict__ st) {
  const int lane = threadIdx.x & 63;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t wave = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nwave = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t tiles = (rows + 15) / 16;
  const float* ub = uv + rl * Fu + VEC * g;
  const int Ffull = F / (4 * VEC) * (4 * VEC);  // blocks fully inside the row
  for (int64_t t = wave; t < tiles; t += nwave) {
    const int64_t row = t * 16 + rl;
    const float* xr = x + (row < rows ? row : rows - 1) * ldx + VEC * g;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    int k0 = 0;
#pragma unroll 4
    for (; k0 < Ffull; k0 += 4 * VEC) {
      float a[VEC], b[VEC];
      if constexpr (VEC == 4) {
        *reinterpret_cast<float4*>(a) = *reinterpret_cast<const float4*>(xr + k0);
        *reinterpret_cast<float4*>(b) = *reinterpret_cast<const float4*>(ub + k0);
      } else if constexpr (VEC == 2) {
        *reinterpret_cast<float2*>(a) = *reinterpret_cast<const float2*>(xr + k0);
        *reinterpret_cast<float2*>(b) = *reinterpret_cast<const float2*>(ub + k0);
      } else {
        a[0] = xr[k0];
        b[0] = ub[k0];
      }
#pragma unroll
      for (int u = 0; u < VEC; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b[u], acc, 0, 0, 0);
    }
    for (; k0 < F; k0 += 4 * VEC) {  // ragged tail: guarded scalar loads
#pragma unroll
      for (int u = 0; u < VEC; ++u) {
        const int f = k0 + VEC * g + u;
        const float xv = xr[(f < F ? f : F - 1) - VEC * g];
        acc = __builtin_amdgcn_mfma_f32_16x16x4f32(f < F ? xv : 0.f, ub[k0 + u], acc, 0, 0, 0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t orow = t * 16 + 4 * g + r;
      if (orow < rows) st[orow * 16 + rl] = acc[r];
    }
  }
}

// Same product with the logit vectors stationary in registers (KSM k-steps of
// 16 features, 4 * KSM VGPRs) and all KSM x loads of a 16-row tile issued
// before the first MFMA: one 16-B load per lane and k-step streams from HBM,
// nothing else.  Rows 16-B aligned (ldx % 4 == 0, x 16-B aligned).
template <int KSM>
__global__ void __launch_bounds__(256) k_logits_s(const float* __restrict__ x, int64_t rows,
                                                  int F, int64_t ldx,
                                                  const float* __restrict__ uv, int Fu,
                                                  float* __restrict__ st,
                                                  float* __restrict__ xmax) {
  const int lane = threadIdx.x & 63;
  const int rl = lane & 15, g = lane >> 4;
  float am = 0.f;  // max |x| over the values this lane loaded (xmax != NULL)
  const int64_t wave = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nwave = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t tiles = (rows + 15) / 16;
  const int ksf = F / 16;                       // k-steps fully inside the row
  const int kst = (F + 15) / 16;                // including the ragged tail
  f32x4 b[KSM];
#pragma unroll
  for (int s = 0; s < KSM; ++s)
    b[s] = s < kst ? *reinterpret_cast<const f32x4*>(uv + rl * Fu + 16 * s + 4 * g)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t t = wave; t < tiles; t += nwave) {
    const int64_t row = t * 16 + rl;
    const float* xr = x + (row < rows ? row : rows - 1) * ldx + 4 * g;
    f32x4 a[KSM];
#pragma unroll
    for (int s = 0; s < KSM; ++s) {
      if (s < ksf) {
        a[s] = *reinterpret_cast<const f32x4*>(xr + 16 * s);
      } else if (s < kst) {  // ragged tail: guarded scalar loads (never past the row)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int f = 16 * s + 4 * g + u;
          a[s][u] = f < F ? xr[16 * s + u] : 0.f;
        }
      } else {
        a[s] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KSM; ++s)
#pragma unroll
      for (int u = 0; u < 4; ++u)
        if (s < kst) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][u], b[s][u], acc, 0, 0, 0);
    if (xmax) {  // clamped tail rows repeat row rows - 1: harmless for a max
#pragma unroll
      for (int s = 0; s < KSM; ++s)
        if (s < kst)
          am = fmaxf(fmaxf(am, fmaxf(fabsf(a[s].x), fabsf(a[s].y))),
                     fmaxf(fabsf(a[s].z), fabsf(a[s].w)));
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int64_t orow = t * 16 + 4 * g + r;
      if (orow < rows) st[orow * 16 + rl] = acc[r];
    }
  }
  if (xmax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
    if (lane == 0)  // non-negative floats order like their bit patterns
      atomicMax(reinterpret_cast<unsigned int*>(xmax), __float_as_uint(am));
  }
}

// max |x| over rows (atomic max into *xmax) for the logits paths that do not
// fold it in (k_logits<VEC>)
__global__ void __launch_bounds__(256) k_absmax(const float* __restrict__ x, int64_t rows, int F,
                                                int64_t ldx, float* __restrict__ xmax) {
  float am = 0.f;
  const int64_t n = rows * int64_t(F);
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t r = i / F;
    am = fmaxf(am, fabsf(x[r * ldx + (i - r * F)]));
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
  if ((threadIdx.x & 63) == 0) atomicMax(reinterpret_cast<unsigned int*>(xmax), __float_as_uint(am));
}

// ---------------------------------------------------------------------------
// One destination segment (or hub chunk) on one wave, single pass with an
// online softmax.  Logit lane layout: lane = 8*k + h (message k of a batch of
// 8, head h); aggregation lane layout: lane <-> feature f = lane + 64q.
// Returns the running max m (head lane & 7) and the denominator reduced over
// the batch lanes; acc[h][q] = sum_j p_jh x_j[f] relative to m.
struct SegState {
  float m;
  float ssum;
};

template <int KF>
__device__ __forceinline__ SegState aggregate_segment(
    const float* __restrict__ x, int64_t ldx, int F, const int32_t* __restrict__ col, int e0,
    int e1, const float* __restrict__ st, float t_h, float slope, float dp, uint64_t seed,
    float (&acc)[H][KF], int j_first = -1) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  const float keep_scale = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) acc[hh][q] = 0.f;
  float m = -INFINITY, l = 0.f;
  for (int b = e0; b < e1; b += 8) {
    const int e = b + kk;
    const bool valid = e < e1;
    // clamped: every load is in bounds; the first batch may come prefetched
    const int j = (b == e0 && j_first >= 0) ? j_first : col[valid ? e : e1 - 1];
    const float v = leaky(st[int64_t(j) * 16 + h] + t_h, slope);
    float bm = valid ? v : -INFINITY;
    bm = fmaxf(bm, __shfl_xor(bm, 8));
    bm = fmaxf(bm, __shfl_xor(bm, 16));
    bm = fmaxf(bm, __shfl_xor(bm, 32));
    const float mn = fmaxf(m, bm);
    const float sc = __expf(m - mn);  // 0 on the first batch, 1 while the max holds
    float p = valid ? __expf(v - mn) : 0.f;
    l = fmaf(l, sc, p);
    if (b != e0 && __any(sc != 1.0f)) {  // wave-uniform: rescale the running sums
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), hh));
#pragma unroll
        for (int q = 0; q < KF; ++q) acc[hh][q] *= s;
      }
    }
    m = mn;
    if (dp > 0.f) p = dropout_keep(seed, uint32_t(e), uint32_t(h), dp) ? p * keep_scale : 0.f;
    const int nk = min(8, e1 - b);
    for (int k0 = 0; k0 < nk; k0 += 4) {  // sub-batches of 4 rows, loads issued together
      float xv[4][KF];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int jk = __builtin_amdgcn_readlane(j, 8 * (k0 + k));
        const float* xr = x + int64_t(jk) * ldx;
#pragma unroll
        for (int q = 0; q < KF; ++q) {
          const int f = lane + 64 * q;
          const float t = xr[f < F ? f : F - 1];
          xv[k][q] = f < F ? t : 0.f;
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
          // p of a padding message is 0: its clamped row adds nothing
          const float pk =
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 8 * (k0 + k) + hh));
#pragma unroll
          for (int q = 0; q < KF; ++q) acc[hh][q] = fmaf(pk, xv[k][q], acc[hh][q]);
        }
      }
    }
  }
  l += __shfl_xor(l, 8);
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  return {m, l};
}

// split 8 fp32 (|v| <= 2^14) into fp16 hi and lo' = (v - hi) * 2^11
__device__ __forceinline__ void split8_f16(const float* v, f16x8& hi, f16x8& lo) {
  union { f16x8 v; _Float16 h[8]; } a, b;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const _Float16 hv = (_Float16)v[j];
    a.h[j] = hv;
    b.h[j] = (_Float16)((v[j] - (float)hv) * kLoScale);
  }
  hi = a.v;
  lo = b.v;
}

__device__ __forceinline__ void mfma_step(const float* __restrict__ Zrow, const uint4& bh,
                                          const uint4& bl, f32x4& acc_m, f32x4& acc_x) {
  float a8[8];
  *reinterpret_cast<float4*>(a8) = *reinterpret_cast<const float4*>(Zrow);
  *reinterpret_cast<float4*>(a8 + 4) = *reinterpret_cast<const float4*>(Zrow + 4);
  f16x8 ahi, alo;
  split8_f16(a8, ahi, alo);
  const f16x8 bhi = *reinterpret_cast<const f16x8*>(&bh);
  const f16x8 blo = *reinterpret_cast<const f16x8*>(&bl);
  acc_m = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bhi, acc_m, 0, 0, 0);
  acc_x = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc_x, 0, 0, 0);
  acc_x = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bhi, acc_x, 0, 0, 0);
}

// same with the A fragment already split (fp16 hi / lo' rows in LDS)
__device__ __forceinline__ void mfma_step_split(const _Float16* __restrict__ zh,
                                                const _Float16* __restrict__ zl, const uint4& bh,
                                                const uint4& bl, f32x4& acc_m, f32x4& acc_x) {
  const f16x8 ahi = *reinterpret_cast<const f16x8*>(zh);
  const f16x8 alo = *reinterpret_cast<const f16x8*>(zl);
  const f16x8 bhi = *reinterpret_cast<const f16x8*>(&bh);
  const f16x8 blo = *reinterpret_cast<const f16x8*>(&bl);
  acc_m = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bhi, acc_m, 0, 0, 0);
  acc_x = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc_x, 0, 0, 0);
  acc_x = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bhi, acc_x, 0, 0, 0);
}

// ---------------------------------------------------------------------------
// Fused tile kernel: 16 destinations per block, one per wave.  The Z tile goes
// through LDS one head-half at a time (16 x 4Fp fp32 = 43 KB at F = 166, two
// blocks per CU).  MFMA work split: column tile ct = w & 3, k-step phase kq = w >> 2;
// the four k-phase partials are summed through LDS at the end.
template <int KF, int OCC>
__global__ void __launch_bounds__(1024, OCC) k_fused(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, int64_t num_dst, int64_t dst_offset,
    const int32_t* __restrict__ order, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ whi,
    const uint4* __restrict__ wlo, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, const int32_t* __restrict__ hub_rank, const float* __restrict__ zhub,
    float* __restrict__ out, float* __restrict__ stats, int mode) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int KH4 = 4 * Fp;                 // K of one head-half
  const int ZS = KH4 + 8;                 // padded row stride (fp16 elements, 16 B pad)
  const int KH = KH4 / 32;                // k-steps per half
  // the half-tile is stored already split: fp16 hi and lo' = (v - hi) * 2^11
  _Float16* Zh = reinterpret_cast<_Float16*>(smem);   // [16][ZS]
  _Float16* Zl = Zh + kTile * ZS;                     // [16][ZS]
  float* red = smem + kTile * ZS;         // [3][4][64][4] k-phase partials
  float* rscale = red + 3 * 4 * 64 * 4;   // [16] per-row 2^-e
  int* rowid = reinterpret_cast<int*>(rscale + kTile);  // [16]
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int64_t slot = int64_t(blockIdx.x) * kTile + wave;
  const int ct = wave & 3, kq = wave >> 2;

  // ---- phase A: this wave's destination, all heads, in registers ----
  float z[H][KF];
  int64_t i = -1;
  int4 dsc = make_int4(-1, 0, 0, -1);
  int j_first = -1;
  if (slot < num_dst) {
    if (desc) {
      // the slot record and its first 8 sources load together: one round trip
      if (cols8) j_first = cols8[slot * 8 + ((threadIdx.x & 63) >> 3)];
      dsc = desc[slot];
    } else {
      const int32_t r = order ? order[slot] : int32_t(slot);
      dsc = make_int4(r, rowptr[r], rowptr[r + 1], hub_rank ? hub_rank[r] : -1);
    }
    i = dsc.x;
  }
  if (mode == 2) {  // ablation: projection only
#pragma unroll
    for (int hh = 0; hh < H; ++hh)
#pragma unroll
      for (int q = 0; q < KF; ++q) z[hh][q] = float(lane + hh + q) * 1e-3f;
  } else if (i >= 0) {
    const int hr = hub_rank ? dsc.w : -1;
    if (hr >= 0) {  // merged (normalised) by k_hub_merge
      const float* src = zhub + int64_t(hr) * (H * Fp);
#pragma unroll
      for (int hh = 0; hh < H; ++hh)
#pragma unroll
        for (int q = 0; q < KF; ++q) {
          const int f = lane + 64 * q;
          z[hh][q] = f < Fp ? src[hh * Fp + f] : 0.f;
        }
    } else {
      const int e0 = dsc.y, e1 = dsc.z;
      const float t_h = st[(dst_offset + i) * 16 + H + (lane & 7)];
      SegState S =
          aggregate_segment<KF>(x, ldx, F, col, e0, e1, st, t_h, slope, dp, seed, z, j_first);
      const float inv_lane = 1.0f / (S.ssum + kSoftmaxEps);
      if (stats && lane < 8) {
        stats[i * 16 + lane] = S.m;
        stats[i * 16 + 8 + lane] = S.ssum;
      }
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inv_lane), hh));
#pragma unroll
        for (int q = 0; q < KF; ++q) z[hh][q] *= inv;
      }
    }
  } else {
#pragma unroll
    for (int hh = 0; hh < H; ++hh)
#pragma unroll
      for (int q = 0; q < KF; ++q) z[hh][q] = 0.f;
  }
  if (mode == 1) {  // ablation: aggregation only
    float sacc = 0.f;
#pragma unroll
    for (int hh = 0; hh < H; ++hh)
#pragma unroll
      for (int q = 0; q < KF; ++q) sacc += z[hh][q];
    if (i >= 0 && lane < C) out[i * C + lane] = sacc;
    return;
  }
  // power-of-two row scale: max |z| -> [2^13, 2^14)
  float zm = 0.f;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) zm = fmaxf(zm, fabsf(z[hh][q]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) zm = fmaxf(zm, __shfl_xor(zm, o));
  int ex = 0;
  if (zm > 0.f) frexpf(zm, &ex);
  int er = 14 - ex;
  er = er > 100 ? 100 : (er < -100 ? -100 : er);
  const float rs = ldexpf(1.0f, er);
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) z[hh][q] *= rs;
  if (lane == 0) {
    rscale[wave] = ldexpf(1.0f, -er);
    rowid[wave] = int(i);
  }

  // ---- phase B over two head-halves ----
  // (addresses below derive from an opaque copy of Fp so that the compiler does
  // not compute them before phase A and hold them through it)
  int Fq = Fp;
  asm volatile("" : "+s"(Fq));
  const int ZSq = 4 * Fq + 8, KHq = Fq / 8;
  const int arow = lane & 15, akg = lane >> 4;
  f32x4 acc_m = {0.f, 0.f, 0.f, 0.f}, acc_x = {0.f, 0.f, 0.f, 0.f};
  _Float16* zrh = Zh + wave * ZSq;
  _Float16* zrl = Zl + wave * ZSq;
#pragma unroll
  for (int hg = 0; hg < 2; ++hg) {
    // W fragments of this wave's first two k-steps: in flight across the barrier
    const int gs0 = hg * KHq;
    uint4 bh0 = {0, 0, 0, 0}, bl0 = {0, 0, 0, 0}, bh1 = {0, 0, 0, 0}, bl1 = {0, 0, 0, 0};
    if (kq < KHq) {
      bh0 = whi[((gs0 + kq) * 4 + ct) * 64 + lane];
      bl0 = wlo[((gs0 + kq) * 4 + ct) * 64 + lane];
    }
    if (kq + 4 < KHq) {
      bh1 = whi[((gs0 + kq + 4) * 4 + ct) * 64 + lane];
      bl1 = wlo[((gs0 + kq + 4) * 4 + ct) * 64 + lane];
    }
    if (hg) __syncthreads();  // half 0 fully consumed
#pragma unroll
    for (int hh = 0; hh < 4; ++hh)
#pragma unroll
      for (int q = 0; q < KF; ++q) {
        const int f = lane + 64 * q;
        if (f < Fq) {
          const float v = z[4 * hg + hh][q];
          const _Float16 hv = (_Float16)v;
          zrh[hh * Fq + f] = hv;
          zrl[hh * Fq + f] = (_Float16)((v - (float)hv) * kLoScale);
        }
      }
    __syncthreads();
    const _Float16* zbh = Zh + arow * ZSq + 8 * akg;
    const _Float16* zbl = Zl + arow * ZSq + 8 * akg;
    for (int s = kq; s < KHq; s += 8) {
      mfma_step_split(zbh + 32 * s, zbl + 32 * s, bh0, bl0, acc_m, acc_x);
      if (s + 8 < KHq) {
        bh0 = whi[((gs0 + s + 8) * 4 + ct) * 64 + lane];
        bl0 = wlo[((gs0 + s + 8) * 4 + ct) * 64 + lane];
      }
      if (s + 4 < KHq) {
        mfma_step_split(zbh + 32 * (s + 4), zbl + 32 * (s + 4), bh1, bl1, acc_m, acc_x);
        if (s + 12 < KHq) {
          bh1 = whi[((gs0 + s + 12) * 4 + ct) * 64 + lane];
          bl1 = wlo[((gs0 + s + 12) * 4 + ct) * 64 + lane];
        }
      }
    }
  }
  f32x4 accv = acc_m + acc_x * (1.0f / kLoScale);
  if (kq) *reinterpret_cast<f32x4*>(red + (((kq - 1) * 4 + ct) * 64 + lane) * 4) = accv;
  __syncthreads();
  if (!kq) {
#pragma unroll
    for (int p = 0; p < 3; ++p)
      accv += *reinterpret_cast<const f32x4*>(red + ((p * 4 + ct) * 64 + lane) * 4);
    const int n = ct * 16 + (lane & 15);
    const float b = bias ? bias[n] : 0.f;
    const float wu = hdr->w_unscale;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (lane >> 4) * 4 + q;
      const int ri = rowid[r];
      if (ri >= 0) out[int64_t(ri) * C + n] = accv[q] * (rscale[r] * wu) + b;
    }
  }
}

// ---------------------------------------------------------------------------
// Weight-stationary persistent tile kernel (one 8-wave block per CU).
//
//  * The projection weights never stream from L2 per tile: each wave keeps the
//    fp16 W_hi B-fragments of its (k-step, column-tile) pairs in VGPRs for the
//    whole launch, and W_lo of the first `nlds` k-steps sits in LDS (the rest
//    is read from L2 just in time).
//  * Two destinations per wave, 16 per tile.  Software pipeline per wave: while
//    tile t's MFMA phase runs, the x rows of tile t+1's first 4 messages (and
//    their logits) are in flight, and tile t+2's slot records are loading.
//  * Z goes through LDS once per head-half, already split into fp16 hi/lo'
//    (so the 4 column-tile waves do not redo the split).
constexpr int kPWaves = 16;

template <int I, int N, typename Fn>
__device__ __forceinline__ void static_for(Fn&& fn) {
  if constexpr (I < N) {
    fn(std::integral_constant<int, I>{});
    static_for<I + 1, N>(fn);
  }
}

struct DstPipe {  // registers of one destination in flight
  int4 d;         // {row, e_begin, e_end, hub_rank}; row < 0 = empty slot
  int j;          // source of message (lane >> 3) of the first batch
};

template <int KF>
struct DstData {
  float th;           // t_i, head lane & 7
  float sj;           // s_j of the lane's first-batch message
  float xv[4][KF];    // x rows of messages 0..3
};

template <int KF>
__device__ __forceinline__ void pipe_rec(DstPipe& p, int64_t slot, int64_t num_dst,
                                         const int4* __restrict__ desc,
                                         const int32_t* __restrict__ cols8) {
  const int kk = (threadIdx.x & 63) >> 3;
  if (slot < num_dst) {
    p.d = desc[slot];
    p.j = cols8 ? cols8[slot * 8 + kk] : -1;
  } else {
    p.d = make_int4(-1, 0, 0, -1);
    p.j = 0;
  }
}

template <int KF>
__device__ __forceinline__ void pipe_issue(DstPipe& p, DstData<KF>& q, const float* __restrict__ x,
                                           int64_t ldx, int F, const int32_t* __restrict__ col,
                                           const float* __restrict__ st, int64_t dst_offset) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  if (p.d.x < 0 || p.d.w >= 0) return;  // empty slot or hub row (merged elsewhere)
  if (p.j < 0) p.j = col[min(p.d.y + kk, p.d.z - 1)];
  q.th = st[(dst_offset + p.d.x) * 16 + H + h];
  q.sj = st[int64_t(p.j) * 16 + h];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int jk = __builtin_amdgcn_readlane(p.j, 8 * k);
    const float* xr = x + int64_t(jk) * ldx;
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) {
      const int f = lane + 64 * qq;
      const float t = xr[f < F ? f : F - 1];
      q.xv[k][qq] = f < F ? t : 0.f;
    }
  }
}

// Aggregate one destination whose first batch is prefetched in (p, q).
template <int KF>
__device__ __forceinline__ void pipe_compute(const DstPipe& p, const DstData<KF>& q,
                                             const float* __restrict__ x, int64_t ldx, int F,
                                             int Fp, const int32_t* __restrict__ col,
                                             const float* __restrict__ st, float slope, float dp,
                                             uint64_t seed, const float* __restrict__ zhub,
                                             float* __restrict__ stats, float (&z)[H][KF]) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) z[hh][qq] = 0.f;
  const int4 d = p.d;
  if (d.x < 0) return;
  if (d.w >= 0) {  // hub: merged row (already normalised)
    const float* src = zhub + int64_t(d.w) * (H * Fp);
#pragma unroll
    for (int hh = 0; hh < H; ++hh)
#pragma unroll
      for (int qq = 0; qq < KF; ++qq) {
        const int f = lane + 64 * qq;
        z[hh][qq] = f < Fp ? src[hh * Fp + f] : 0.f;
      }
    return;
  }
  const int e0 = p.d.y, e1 = p.d.z;
  const float keep_scale = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
  float m = -INFINITY, l = 0.f;
  for (int b = e0; b < e1; b += 8) {
    const int e = b + kk;
    const bool valid = e < e1;
    int j;
    float v;
    if (b == e0) {
      j = p.j;
      v = leaky(q.sj + q.th, slope);
    } else {
      j = col[valid ? e : e1 - 1];
      v = leaky(st[int64_t(j) * 16 + h] + q.th, slope);
    }
    float bm = valid ? v : -INFINITY;
    bm = fmaxf(bm, __shfl_xor(bm, 8));
    bm = fmaxf(bm, __shfl_xor(bm, 16));
    bm = fmaxf(bm, __shfl_xor(bm, 32));
    const float mn = fmaxf(m, bm);
    const float sc = __expf(m - mn);
    float pv = valid ? __expf(v - mn) : 0.f;
    l = fmaf(l, sc, pv);
    if (b != e0 && __any(sc != 1.0f)) {
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), hh));
#pragma unroll
        for (int qq = 0; qq < KF; ++qq) z[hh][qq] *= s;
      }
    }
    m = mn;
    if (dp > 0.f) pv = dropout_keep(seed, uint32_t(e), uint32_t(h), dp) ? pv * keep_scale : 0.f;
    const int nk = min(8, e1 - b);
    for (int k0 = 0; k0 < nk; k0 += 4) {
      float xl[4][KF];
      if (b == e0 && k0 == 0) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
#pragma unroll
          for (int qq = 0; qq < KF; ++qq) xl[k][qq] = q.xv[k][qq];
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const int jk = __builtin_amdgcn_readlane(j, 8 * (k0 + k));
          const float* xr = x + int64_t(jk) * ldx;
#pragma unroll
          for (int qq = 0; qq < KF; ++qq) {
            const int f = lane + 64 * qq;
            const float t = xr[f < F ? f : F - 1];
            xl[k][qq] = f < F ? t : 0.f;
          }
        }
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
          const float pk =
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), 8 * (k0 + k) + hh));
#pragma unroll
          for (int qq = 0; qq < KF; ++qq) z[hh][qq] = fmaf(pk, xl[k][qq], z[hh][qq]);
        }
    }
  }
  l += __shfl_xor(l, 8);
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  if (stats && lane < 8) {
    stats[int64_t(d.x) * 16 + lane] = m;
    stats[int64_t(d.x) * 16 + 8 + lane] = l;
  }
  const float inv_lane = 1.0f / (l + kSoftmaxEps);
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inv_lane), hh));
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) z[hh][qq] *= inv;
  }
}

// power-of-two row scale so that max |z| lies in [2^13, 2^14); returns 2^-e
template <int KF>
__device__ __forceinline__ float scale_row(float (&z)[H][KF]) {
  float zm = 0.f;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) zm = fmaxf(zm, fabsf(z[hh][q]));
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) zm = fmaxf(zm, __shfl_xor(zm, o));
  int ex = 0;
  if (zm > 0.f) frexpf(zm, &ex);
  int er = 14 - ex;
  er = er > 100 ? 100 : (er < -100 ? -100 : er);
  const float rs = ldexpf(1.0f, er);
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) z[hh][q] *= rs;
  return ldexpf(1.0f, -er);
}

// write heads [4*hg, 4*hg+4) of one row into the half-tile as fp16 hi / lo'
template <int KF>
__device__ __forceinline__ void write_half(const float (&z)[H][KF], int hg, int Fp,
                                           _Float16* __restrict__ zh, _Float16* __restrict__ zl) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int hh = 0; hh < 4; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) {
      const int f = lane + 64 * q;
      if (f < Fp) {
        const float v = z[4 * hg + hh][q];
        const _Float16 hv = (_Float16)v;
        zh[hh * Fp + f] = hv;
        zl[hh * Fp + f] = (_Float16)((v - (float)hv) * kLoScale);
      }
    }
}

// 16 waves, one destination per wave and tile; wave (ct = w & 3, kq = w >> 2)
// owns the MFMA k-steps s = kq + 4u (u < NKW) of column tile ct: their W_hi
// fragments live in VGPRs for the whole launch, W_lo of k-steps s < nl in LDS,
// the rest of W_lo streams from L2 (nl is as large as the LDS allows).
template <int KF, int NKW>
__global__ void __launch_bounds__(kPWaves * 64, 4) k_persist(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ whi,
    const uint4* __restrict__ wlo, int nl, const float* __restrict__ bias, float slope,
    float dp, uint64_t seed, const float* __restrict__ zhub, float* __restrict__ out,
    float* __restrict__ stats, int64_t num_tiles) {
  extern __shared__ __attribute__((aligned(16))) char psm[];
  const int KH4 = 4 * Fp;           // K of a head-half (multiple of 32)
  const int KH = KH4 / 32;          // k-steps per half
  const int KS = 2 * KH;
  const int ZS = KH4 + 8;           // half-tile row stride in fp16 (16-B pad)
  _Float16* Zh = reinterpret_cast<_Float16*>(psm);            // [16][ZS]
  _Float16* Zl = Zh + kTile * ZS;                             // [16][ZS]
  float* red = reinterpret_cast<float*>(Zl + kTile * ZS);     // [3][4][64][4]
  float* rsc0 = red + 3 * 4 * 64 * 4;                         // [2][16] by tile parity
  int* rid0 = reinterpret_cast<int*>(rsc0 + 2 * kTile);       // [2][16]
  uint4* WL = reinterpret_cast<uint4*>(rid0 + 2 * kTile);     // [nl][4][64]

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = wave_uniform(tid >> 6);
  const int ct = wave & 3, kq = wave >> 2;
  const int arow = lane & 15, akg = lane >> 4;

  uint4 wh[NKW];
#pragma unroll
  for (int u = 0; u < NKW; ++u) {
    const int s = kq + 4 * u;
    wh[u] = s < KS ? whi[(s * 4 + ct) * 64 + lane] : make_uint4(0, 0, 0, 0);
  }
  for (int idx = tid; idx < nl * 256; idx += kPWaves * 64) WL[idx] = wlo[idx];
  const float wu = hdr->w_unscale;
  const float bcol = bias ? bias[ct * 16 + (lane & 15)] : 0.f;

  DstPipe pc, pn;
  DstData<KF> dd;
  int64_t t = blockIdx.x;
  const int64_t G = gridDim.x;
  pipe_rec<KF>(pc, t * kTile + wave, num_dst, desc, cols8);
  pipe_issue<KF>(pc, dd, x, ldx, F, col, st, dst_offset);
  pipe_rec<KF>(pn, (t + G) * kTile + wave, num_dst, desc, cols8);
  __syncthreads();  // WL ready

  for (int it = 0; t < num_tiles; t += G, ++it) {
    // An opaque per-tile copy of the row width: every address derived from it is
    // recomputed inside the loop instead of being hoisted and held in VGPRs
    // across the whole launch (the compiler's LICM otherwise pins ~50 VGPRs of
    // 64-bit per-head offsets).
    int Fq = Fp;
    asm volatile("" : "+s"(Fq));
    const int KHq = Fq / 8;  // k-steps per head-half (4 * Fq / 32)
    const int ZSq = 4 * Fq + 8;
    float* rsc = rsc0 + (it & 1) * kTile;
    int* rid = rid0 + (it & 1) * kTile;
    // ---- phase A: this wave's destination; next tile's first batch then in flight ----
    float z[H][KF];
    pipe_compute<KF>(pc, dd, x, ldx, F, Fq, col, st, slope, dp, seed, zhub, stats, z);
    const int ri = pc.d.x;
    pc = pn;
    pipe_issue<KF>(pc, dd, x, ldx, F, col, st, dst_offset);
    pipe_rec<KF>(pn, (t + 2 * G) * kTile + wave, num_dst, desc, cols8);
    const float sr = scale_row<KF>(z);
    if (lane == 0) {
      rsc[wave] = sr;
      rid[wave] = ri;
    }
    // ---- phase B: out[16 x 64] = Z . Wcat, one head-half at a time ----
    f32x4 acc_m = {0.f, 0.f, 0.f, 0.f}, acc_x = {0.f, 0.f, 0.f, 0.f};
    const _Float16* ah = Zh + arow * ZSq + 8 * akg;
    const _Float16* al = Zl + arow * ZSq + 8 * akg;
    int wofs = (kq * 4 + ct) * 64 + lane;  // fragment index of k-step kq; +1024 per u
    asm volatile("" : "+v"(wofs));
#pragma unroll
    for (int hg = 0; hg < 2; ++hg) {
      if (hg) __syncthreads();  // half 0 consumed
      write_half<KF>(z, hg, Fq, Zh + wave * ZSq, Zl + wave * ZSq);
      __syncthreads();
      static_for<0, NKW>([&](auto ui) {
        constexpr int u = decltype(ui)::value;
        const int s = kq + 4 * u;
        if (s < 2 * KHq && (s >= KHq) == (hg == 1)) {
          const int ko = 32 * (s - hg * KHq);
          const uint4 blo = s < nl ? WL[wofs + 1024 * u] : wlo[wofs + 1024 * u];
          const f16x8 a_hi = *reinterpret_cast<const f16x8*>(ah + ko);
          const f16x8 a_lo = *reinterpret_cast<const f16x8*>(al + ko);
          const f16x8 b_hi = *reinterpret_cast<const f16x8*>(&wh[u]);
          const f16x8 b_lo = *reinterpret_cast<const f16x8*>(&blo);
          acc_m = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi, b_hi, acc_m, 0, 0, 0);
          acc_x = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_hi, b_lo, acc_x, 0, 0, 0);
          acc_x = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_lo, b_hi, acc_x, 0, 0, 0);
        }
      });
    }
    f32x4 accv = acc_m + acc_x * (1.0f / kLoScale);
    if (kq) *reinterpret_cast<f32x4*>(red + (((kq - 1) * 4 + ct) * 64 + lane) * 4) = accv;
    __syncthreads();  // partials visible; every read of this tile's half 1 done
    if (!kq) {
#pragma unroll
      for (int pp = 0; pp < 3; ++pp)
        accv += *reinterpret_cast<const f32x4*>(red + ((pp * 4 + ct) * 64 + lane) * 4);
      const int n = ct * 16 + (lane & 15);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int r = (lane >> 4) * 4 + q;
        const int rr = rid[r];
        if (rr >= 0) out[int64_t(rr) * C + n] = accv[q] * (rsc[r] * wu) + bcol;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Phase A of one tile slot: the normalised z of the slot's destination (all 8
// heads, fp32, lane <-> feature) or zeros for an empty slot.  Returns the
// destination row (or -1).
template <int KF>
__device__ __forceinline__ int slot_aggregate(
    int64_t slot, int64_t num_dst, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ x, int64_t ldx, int F, int Fp,
    const int32_t* __restrict__ col, int64_t dst_offset, const float* __restrict__ st,
    float slope, float dp, uint64_t seed, const float* __restrict__ zhub,
    float* __restrict__ stats, float (&z)[H][KF]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) z[hh][q] = 0.f;
  if (slot >= num_dst) return -1;
  const int j_first = cols8 ? cols8[slot * 8 + (lane >> 3)] : -1;
  const int4 dsc = desc[slot];
  const int i = dsc.x;
  if (dsc.w >= 0) {  // hub: merged, normalised row from k_hub_merge
    const float* src = zhub + int64_t(dsc.w) * (H * Fp);
#pragma unroll
    for (int hh = 0; hh < H; ++hh)
#pragma unroll
      for (int q = 0; q < KF; ++q) {
        const int f = lane + 64 * q;
        z[hh][q] = f < Fp ? src[hh * Fp + f] : 0.f;
      }
    return i;
  }
  const float t_h = st[(dst_offset + i) * 16 + H + (lane & 7)];
  SegState S =
      aggregate_segment<KF>(x, ldx, F, col, dsc.y, dsc.z, st, t_h, slope, dp, seed, z, j_first);
  const float inv_lane = 1.0f / (S.ssum + kSoftmaxEps);
  if (stats && lane < 8) {
    stats[int64_t(i) * 16 + lane] = S.m;
    stats[int64_t(i) * 16 + 8 + lane] = S.ssum;
  }
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inv_lane), hh));
#pragma unroll
    for (int q = 0; q < KF; ++q) z[hh][q] *= inv;
  }
  return i;
}

// ---------------------------------------------------------------------------
// 32-row tile kernel: 16 waves, two destinations per wave (rows w and w + 16),
// so each W fragment streamed from L2 feeds two MFMA row blocks (344 KB of
// W per 32 destinations at F = 166 instead of per 16).  The half-tile
// (32 x 4Fp, fp16 hi/lo) is 87 KB: one block per CU.  Heads 4-7 of both rows
// wait in registers while half 0 is projected.
template <int KF>
__global__ void __launch_bounds__(1024, 4) k_tile32(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ whi,
    const uint4* __restrict__ wlo, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, const float* __restrict__ zhub, float* __restrict__ out,
    float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int ct = wave & 3, kq = wave >> 2;
  const int64_t base = int64_t(blockIdx.x) * 32;

  // ---- phase A: rows wave and wave + 16 ----
  float zk[2][4][KF];  // heads 4..7 of both rows, scaled
  int rows[2];
  float rsc[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    float z[H][KF];
    rows[d] = slot_aggregate<KF>(base + wave + 16 * d, num_dst, desc, cols8, x, ldx, F, Fp, col,
                                 dst_offset, st, slope, dp, seed, zhub, stats, z);
    rsc[d] = scale_row<KF>(z);
    int Fq = Fp;
    asm volatile("" : "+s"(Fq));
    const int ZSq = 4 * Fq + 8;
    _Float16* Zh = reinterpret_cast<_Float16*>(smem);
    write_half<KF>(z, 0, Fq, Zh + (wave + 16 * d) * ZSq, Zh + (32 + wave + 16 * d) * ZSq);
#pragma unroll
    for (int hh = 0; hh < 4; ++hh)
#pragma unroll
      for (int q = 0; q < KF; ++q) zk[d][hh][q] = z[4 + hh][q];
  }
  int Fq = Fp;
  asm volatile("" : "+s"(Fq));
  const int ZSq = 4 * Fq + 8, KHq = Fq / 8;
  _Float16* Zh = reinterpret_cast<_Float16*>(smem);    // [32][ZS]
  _Float16* Zl = Zh + 32 * ZSq;                        // [32][ZS]
  float* red = reinterpret_cast<float*>(Zl + 32 * ZSq);  // [3][4][64][8]
  float* rscale = red + 3 * 4 * 64 * 8;                // [32]
  int* rowid = reinterpret_cast<int*>(rscale + 32);    // [32]
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      rscale[wave + 16 * d] = rsc[d];
      rowid[wave + 16 * d] = rows[d];
    }
  }

  // ---- phase B: out[32 x 64] = Z . Wcat, two head-halves ----
  const int arow = lane & 15, akg = lane >> 4;
  f32x4 am0 = {0.f, 0.f, 0.f, 0.f}, ax0 = am0, am1 = am0, ax1 = am0;
  const _Float16* zb0 = Zh + arow * ZSq + 8 * akg;
  const _Float16* zl0 = Zl + arow * ZSq + 8 * akg;
  const _Float16* zb1 = zb0 + 16 * ZSq;
  const _Float16* zl1 = zl0 + 16 * ZSq;
#pragma unroll
  for (int hg = 0; hg < 2; ++hg) {
    const int gs0 = hg * KHq;
    uint4 bh = {0, 0, 0, 0}, bl = {0, 0, 0, 0};
    if (kq < KHq) {
      bh = whi[((gs0 + kq) * 4 + ct) * 64 + lane];
      bl = wlo[((gs0 + kq) * 4 + ct) * 64 + lane];
    }
    if (hg) {
      __syncthreads();  // half 0 fully consumed
#pragma unroll
      for (int d = 0; d < 2; ++d) {
        const int r = wave + 16 * d;
#pragma unroll
        for (int hh = 0; hh < 4; ++hh)
#pragma unroll
          for (int q = 0; q < KF; ++q) {
            const int f = lane + 64 * q;
            if (f < Fq) {
              const float v = zk[d][hh][q];
              const _Float16 hv = (_Float16)v;
              Zh[r * ZSq + hh * Fq + f] = hv;
              Zl[r * ZSq + hh * Fq + f] = (_Float16)((v - (float)hv) * kLoScale);
            }
          }
      }
    }
    __syncthreads();
    for (int s = kq; s < KHq; s += 4) {
      uint4 nh = {0, 0, 0, 0}, nlo = {0, 0, 0, 0};
      if (s + 4 < KHq) {
        nh = whi[((gs0 + s + 4) * 4 + ct) * 64 + lane];
        nlo = wlo[((gs0 + s + 4) * 4 + ct) * 64 + lane];
      }
      const f16x8 bhi = *reinterpret_cast<const f16x8*>(&bh);
      const f16x8 blo = *reinterpret_cast<const f16x8*>(&bl);
      const f16x8 a0h = *reinterpret_cast<const f16x8*>(zb0 + 32 * s);
      const f16x8 a0l = *reinterpret_cast<const f16x8*>(zl0 + 32 * s);
      const f16x8 a1h = *reinterpret_cast<const f16x8*>(zb1 + 32 * s);
      const f16x8 a1l = *reinterpret_cast<const f16x8*>(zl1 + 32 * s);
      am0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, bhi, am0, 0, 0, 0);
      am1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1h, bhi, am1, 0, 0, 0);
      ax0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, blo, ax0, 0, 0, 0);
      ax1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1h, blo, ax1, 0, 0, 0);
      ax0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0l, bhi, ax0, 0, 0, 0);
      ax1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1l, bhi, ax1, 0, 0, 0);
      bh = nh;
      bl = nlo;
    }
  }
  f32x4 acc0 = am0 + ax0 * (1.0f / kLoScale);
  f32x4 acc1 = am1 + ax1 * (1.0f / kLoScale);
  if (kq) {
    float* rp = red + (((kq - 1) * 4 + ct) * 64 + lane) * 8;
    *reinterpret_cast<f32x4*>(rp) = acc0;
    *reinterpret_cast<f32x4*>(rp + 4) = acc1;
  }
  __syncthreads();
  if (!kq) {
#pragma unroll
    for (int pp = 0; pp < 3; ++pp) {
      const float* rp = red + ((pp * 4 + ct) * 64 + lane) * 8;
      acc0 += *reinterpret_cast<const f32x4*>(rp);
      acc1 += *reinterpret_cast<const f32x4*>(rp + 4);
    }
    const int n = ct * 16 + (lane & 15);
    const float b = bias ? bias[n] : 0.f;
    const float wu = hdr->w_unscale;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (lane >> 4) * 4 + q;
      const int r0 = rowid[r], r1 = rowid[16 + r];
      if (r0 >= 0) out[int64_t(r0) * C + n] = acc0[q] * (rscale[r] * wu) + b;
      if (r1 >= 0) out[int64_t(r1) * C + n] = acc1[q] * (rscale[16 + r] * wu) + b;
    }
  }
}

// ---------------------------------------------------------------------------
// Two destinations aggregated concurrently by one wave: both slot records and
// first-batch columns load in one round trip, both first batches of x rows in
// the next, so twice the rows are in flight per wave compared with
// aggregate_segment.  Same arithmetic per destination as aggregate_segment
// (online softmax over batches of 8 messages, rows in sub-batches of 4).
template <int KF>
struct PairSeg {
  int e0, n;    // CSR start and message count (n = 0: nothing to aggregate)
  int jf;       // prefetched column of message (lane >> 3) of the first batch, or -1
  float t;      // t_i for head lane & 7
  float m, l;   // running max (head lane & 7), running denominator (per lane)
};

template <int KF>
__device__ __forceinline__ void pair_logits(PairSeg<KF>& S, int b, bool first,
                                            const int32_t* __restrict__ col,
                                            const float* __restrict__ st, float slope, float dp,
                                            uint64_t seed, float (&z)[H][KF], int& j, float& p) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  const bool valid = b + kk < S.n;
  const int e = S.e0 + min(b + kk, S.n - 1);
  j = (first && S.jf >= 0) ? S.jf : col[e];
  const float v = leaky(st[int64_t(j) * 16 + h] + S.t, slope);
  float bm = valid ? v : -INFINITY;
  bm = fmaxf(bm, __shfl_xor(bm, 8));
  bm = fmaxf(bm, __shfl_xor(bm, 16));
  bm = fmaxf(bm, __shfl_xor(bm, 32));
  const float mn = fmaxf(S.m, bm);
  const float sc = __expf(S.m - mn);
  p = valid ? __expf(v - mn) : 0.f;
  S.l = fmaf(S.l, sc, p);
  if (!first && __any(sc != 1.0f)) {
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
      const float s = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), hh));
#pragma unroll
      for (int q = 0; q < KF; ++q) z[hh][q] *= s;
    }
  }
  S.m = mn;
  if (dp > 0.f)
    p = dropout_keep(seed, uint32_t(S.e0 + b + kk), uint32_t(h), dp) ? p * (1.0f / (1.0f - dp)) : 0.f;
}

template <int KF>
__device__ __forceinline__ void pair_rows(const float* __restrict__ x, int64_t ldx, int F, int j,
                                          int k0, float (&xv)[4][KF]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int jk = __builtin_amdgcn_readlane(j, 8 * (k0 + k));
    const float* xr = x + int64_t(jk) * ldx;
#pragma unroll
    for (int q = 0; q < KF; ++q) {
      const int f = lane + 64 * q;
      const float t = xr[f < F ? f : F - 1];
      xv[k][q] = f < F ? t : 0.f;
    }
  }
}

template <int KF>
__device__ __forceinline__ void pair_fma(float p, int k0, const float (&xv)[4][KF],
                                         float (&z)[H][KF]) {
#pragma unroll
  for (int k = 0; k < 4; ++k)
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
      const float pk = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 8 * (k0 + k) + hh));
#pragma unroll
      for (int q = 0; q < KF; ++q) z[hh][q] = fmaf(pk, xv[k][q], z[hh][q]);
    }
}

// 32-row tiles (rows w and w + 16 of a tile go to wave w) with both rows'
// aggregation interleaved; phase B as k_tile32.
template <int KF>
__global__ void __launch_bounds__(1024, 4) k_pair(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ whi,
    const uint4* __restrict__ wlo, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, const float* __restrict__ zhub, float* __restrict__ out,
    float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int ct = wave & 3, kq = wave >> 2;
  const int64_t base = int64_t(blockIdx.x) * 32;

  // ---- phase A: rows wave (a) and wave + 16 (b), interleaved ----
  float za[H][KF], zb[H][KF];
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) za[hh][q] = zb[hh][q] = 0.f;
  const int64_t sa = base + wave, sb = base + wave + 16;
  int4 da = make_int4(-1, 0, 0, -1), db = make_int4(-1, 0, 0, -1);
  PairSeg<KF> A, B;
  A.jf = B.jf = -1;
  if (sa < num_dst) {
    if (cols8) A.jf = cols8[sa * 8 + (lane >> 3)];
    da = desc[sa];
  }
  if (sb < num_dst) {
    if (cols8) B.jf = cols8[sb * 8 + (lane >> 3)];
    db = desc[sb];
  }
  const bool agg_a = da.x >= 0 && da.w < 0, agg_b = db.x >= 0 && db.w < 0;
  A.e0 = da.y; A.n = agg_a ? da.z - da.y : 0;
  B.e0 = db.y; B.n = agg_b ? db.z - db.y : 0;
  A.t = agg_a ? st[(dst_offset + da.x) * 16 + H + (lane & 7)] : 0.f;
  B.t = agg_b ? st[(dst_offset + db.x) * 16 + H + (lane & 7)] : 0.f;
  A.m = B.m = -INFINITY;
  A.l = B.l = 0.f;
  const int len = max(A.n, B.n);
  for (int b = 0; b < len; b += 8) {
    const bool first = b == 0;
    const bool act_a = b < A.n, act_b = b < B.n;
    int ja = 0, jb = 0;
    float pa = 0.f, pb = 0.f;
    if (act_a) pair_logits<KF>(A, b, first, col, st, slope, dp, seed, za, ja, pa);
    if (act_b) pair_logits<KF>(B, b, first, col, st, slope, dp, seed, zb, jb, pb);
    const int nka = act_a ? min(8, A.n - b) : 0, nkb = act_b ? min(8, B.n - b) : 0;
    for (int k0 = 0; k0 < max(nka, nkb); k0 += 4) {
      float xa[4][KF], xb[4][KF];
      if (k0 < nka) pair_rows<KF>(x, ldx, F, ja, k0, xa);
      if (k0 < nkb) pair_rows<KF>(x, ldx, F, jb, k0, xb);
      if (k0 < nka) pair_fma<KF>(pa, k0, xa, za);
      if (k0 < nkb) pair_fma<KF>(pb, k0, xb, zb);
    }
  }
  int rows[2] = {da.x, db.x};
  float rsc[2];
#pragma unroll
  for (int d = 0; d < 2; ++d) {
    float (&z)[H][KF] = d ? zb : za;
    const int4 dd = d ? db : da;
    PairSeg<KF>& S = d ? B : A;
    if (dd.x >= 0 && dd.w >= 0) {  // hub: merged, normalised row
      int Fq = Fp;
      asm volatile("" : "+s"(Fq));
      const float* src = zhub + int64_t(dd.w) * (H * Fq);
#pragma unroll
      for (int hh = 0; hh < H; ++hh)
#pragma unroll
        for (int q = 0; q < KF; ++q) {
          const int f = lane + 64 * q;
          z[hh][q] = f < Fq ? src[hh * Fq + f] : 0.f;
        }
    } else if (dd.x >= 0) {
      float l = S.l;
      l += __shfl_xor(l, 8);
      l += __shfl_xor(l, 16);
      l += __shfl_xor(l, 32);
      if (stats && lane < 8) {
        stats[int64_t(dd.x) * 16 + lane] = S.m;
        stats[int64_t(dd.x) * 16 + 8 + lane] = l;
      }
      const float inv_lane = 1.0f / (l + kSoftmaxEps);
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inv_lane), hh));
#pragma unroll
        for (int q = 0; q < KF; ++q) z[hh][q] *= inv;
      }
    }
    rsc[d] = scale_row<KF>(z);
  }
  int Fq = Fp;
  asm volatile("" : "+s"(Fq));
  const int ZSq = 4 * Fq + 8, KHq = Fq / 8;
  _Float16* Zh = reinterpret_cast<_Float16*>(smem);    // [32][ZS]
  _Float16* Zl = Zh + 32 * ZSq;                        // [32][ZS]
  float* red = reinterpret_cast<float*>(Zl + 32 * ZSq);  // [3][4][64][8]
  float* rscale = red + 3 * 4 * 64 * 8;                // [32]
  int* rowid = reinterpret_cast<int*>(rscale + 32);    // [32]
  write_half<KF>(za, 0, Fq, Zh + wave * ZSq, Zl + wave * ZSq);
  write_half<KF>(zb, 0, Fq, Zh + (wave + 16) * ZSq, Zl + (wave + 16) * ZSq);
  if (lane == 0) {
#pragma unroll
    for (int d = 0; d < 2; ++d) {
      rscale[wave + 16 * d] = rsc[d];
      rowid[wave + 16 * d] = rows[d];
    }
  }

  // ---- phase B: out[32 x 64] = Z . Wcat, two head-halves ----
  const int arow = lane & 15, akg = lane >> 4;
  f32x4 am0 = {0.f, 0.f, 0.f, 0.f}, ax0 = am0, am1 = am0, ax1 = am0;
  const _Float16* zb0 = Zh + arow * ZSq + 8 * akg;
  const _Float16* zl0 = Zl + arow * ZSq + 8 * akg;
  const _Float16* zb1 = zb0 + 16 * ZSq;
  const _Float16* zl1 = zl0 + 16 * ZSq;
#pragma unroll
  for (int hg = 0; hg < 2; ++hg) {
    const int gs0 = hg * KHq;
    uint4 bh = {0, 0, 0, 0}, bl = {0, 0, 0, 0};
    if (kq < KHq) {
      bh = whi[((gs0 + kq) * 4 + ct) * 64 + lane];
      bl = wlo[((gs0 + kq) * 4 + ct) * 64 + lane];
    }
    if (hg) {
      __syncthreads();  // half 0 fully consumed
      write_half<KF>(za, 1, Fq, Zh + wave * ZSq, Zl + wave * ZSq);
      write_half<KF>(zb, 1, Fq, Zh + (wave + 16) * ZSq, Zl + (wave + 16) * ZSq);
    }
    __syncthreads();
    for (int s = kq; s < KHq; s += 4) {
      uint4 nh = {0, 0, 0, 0}, nlo = {0, 0, 0, 0};
      if (s + 4 < KHq) {
        nh = whi[((gs0 + s + 4) * 4 + ct) * 64 + lane];
        nlo = wlo[((gs0 + s + 4) * 4 + ct) * 64 + lane];
      }
      const f16x8 bhi = *reinterpret_cast<const f16x8*>(&bh);
      const f16x8 blo = *reinterpret_cast<const f16x8*>(&bl);
      const f16x8 a0h = *reinterpret_cast<const f16x8*>(zb0 + 32 * s);
      const f16x8 a0l = *reinterpret_cast<const f16x8*>(zl0 + 32 * s);
      const f16x8 a1h = *reinterpret_cast<const f16x8*>(zb1 + 32 * s);
      const f16x8 a1l = *reinterpret_cast<const f16x8*>(zl1 + 32 * s);
      am0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, bhi, am0, 0, 0, 0);
      am1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1h, bhi, am1, 0, 0, 0);
      ax0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0h, blo, ax0, 0, 0, 0);
      ax1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1h, blo, ax1, 0, 0, 0);
      ax0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0l, bhi, ax0, 0, 0, 0);
      ax1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1l, bhi, ax1, 0, 0, 0);
      bh = nh;
      bl = nlo;
    }
  }
  f32x4 acc0 = am0 + ax0 * (1.0f / kLoScale);
  f32x4 acc1 = am1 + ax1 * (1.0f / kLoScale);
  if (kq) {
    float* rp = red + (((kq - 1) * 4 + ct) * 64 + lane) * 8;
    *reinterpret_cast<f32x4*>(rp) = acc0;
    *reinterpret_cast<f32x4*>(rp + 4) = acc1;
  }
  __syncthreads();
  if (!kq) {
#pragma unroll
    for (int pp = 0; pp < 3; ++pp) {
      const float* rp = red + ((pp * 4 + ct) * 64 + lane) * 8;
      acc0 += *reinterpret_cast<const f32x4*>(rp);
      acc1 += *reinterpret_cast<const f32x4*>(rp + 4);
    }
    const int n = ct * 16 + (lane & 15);
    const float bb = bias ? bias[n] : 0.f;
    const float wu = hdr->w_unscale;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (lane >> 4) * 4 + q;
      const int r0 = rowid[r], r1 = rowid[16 + r];
      if (r0 >= 0) out[int64_t(r0) * C + n] = acc0[q] * (rscale[r] * wu) + bb;
      if (r1 >= 0) out[int64_t(r1) * C + n] = acc1[q] * (rscale[16 + r] * wu) + bb;
    }
  }
}


// ---------------------------------------------------------------------------
// k_stream and its slot helpers (kernel comment below).
constexpr int kSWaves = 8;
#ifndef GFD_STREAM_AP_LIGHT  // the same for the light-tile kernel (fewer live registers)
#define GFD_STREAM_AP_LIGHT 2
#endif
#ifndef GFD_STREAM_AP  // A-fragment k-steps read ahead in the MFMA loop
#define GFD_STREAM_AP 2
#endif
// k_stream phase ablation for diagnostic builds (-DGFD_STREAM_ABLATE=1: no MFMA,
// 2: no aggregation); compile-time so the product kernel carries no branch
#ifdef GFD_STREAM_ABLATE
constexpr int kAblate = GFD_STREAM_ABLATE;
#else
constexpr int kAblate = 0;
#endif

#ifdef GFD_CHECKED
// Checked diagnostic build (-DGFD_CHECKED): every gathered index of k_stream is
// bounds-checked; the first violation is recorded (site, value, limit, block)
// and the index replaced by 0, so a bad index reports instead of faulting.
__device__ long long g_chk[4];
__device__ long long g_lim[4];  // x/st rows (N), num_dst, num_hubs
__device__ __noinline__ void chk_fail(int site, long long v, long long lim) {
  if (atomicCAS(reinterpret_cast<unsigned long long*>(&g_chk[0]), 0ull,
                (unsigned long long)site) == 0ull) {
    g_chk[1] = v;
    g_chk[2] = lim;
    g_chk[3] = blockIdx.x * 1000 + (threadIdx.x >> 6);
  }
}
#define CHK(site, v, limi) \
  ((unsigned long long)(v) < (unsigned long long)g_lim[limi] ? (v) : (chk_fail(site, (v), g_lim[limi]), 0))
#else
#define CHK(site, v, limi) (v)
#endif

#ifdef GFD_PROF
// Phase cycle counters of k_stream (diagnostic builds only, -DGFD_PROF):
// 0 MFMA, 1 barrier after MFMA, 2 reduce+store, 3 aggregate slot 0,
// 4 aggregate slot 1, 5 issue+records, 6 barrier after aggregation, 7 tiles
constexpr int kProfN = 32;
__device__ unsigned long long g_prof[kProfN];
#define PROF_MARK(i)                                                              \
  do {                                                                            \
    const uint64_t t_ = __builtin_readcyclecounter();                             \
    if ((threadIdx.x & 63) == 0) prof_lds[(threadIdx.x >> 6) * kProfN + (i)] += uint32_t(t_ - prof_t); \
    prof_t = t_;                                                                  \
  } while (0)
#define PROF_PARAMS , uint64_t &prof_t, uint32_t *prof_lds
#define PROF_PASS , prof_t, prof_lds
#else
#define PROF_MARK(i)
#define PROF_PARAMS
#define PROF_PASS
#endif

// The stream kernel's helpers take the lane index as an argument: the kernel
// launders it (asm) once per tile, so no per-lane address derived from it can
// be hoisted out of the persistent loop and pinned in VGPRs for the whole
// launch (the registers belong to the stationary weights).
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

struct SlotRec {  // one tile slot as loaded (vector loads: no SMEM in the lgkm queue)
  int v;          // lanes 0..3: {row, e_begin, e_end, hub_rank}; lanes 8..15: sources of
                  // messages 0..7 (slot_cols); other lanes: row
  bool live;      // slot < num_dst (otherwise v is a clamped copy, row taken as -1)
};

__device__ __forceinline__ int4 uni4(int4 v) {
  return make_int4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                   __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}

struct SlotRing {  // the same record parked in LDS between issue and aggregation
  int4 d;
  int j[8];
};

template <int KF, int PFN = 4>
struct SlotRows {  // first batch in flight
  static constexpr int PF = PFN;  // rows issued ahead (register budget)
  float th;        // t_i of head lane & 7
  float sj;        // s_j of the lane's message
  int cj;          // source of message 8 + lane (0 past the end; nothing fetched for <= 8)
  float xv[PF][KF];  // x rows of messages 0..PF-1 (lane <-> feature)
};

__device__ __forceinline__ void sl_rec(SlotRec& p, int64_t slot, int64_t num_dst,
                                       const int4* __restrict__ desc,
                                       const int32_t* __restrict__ cols8, int lane) {
  const int64_t sl = slot < num_dst ? slot : num_dst - 1;
  const int32_t* a = reinterpret_cast<const int32_t*>(desc + CHK(1, sl, 1)) + (lane & 3);
  const int32_t* b = cols8 + CHK(2, sl, 1) * 8 + (lane & 7);
  p.v = *((lane & 56) == 8 ? b : a);  // one dword per lane, one VGPR per slot
  p.live = slot < num_dst;
}

// x row j: an unsigned 32 x 32 -> 64-bit product (two scalar multiplies) instead
// of a sign-extended 64-bit one (the scalar unit is shared by the CU's waves);
// j >= 0 and 4 * ldx < 2^32 (checked on the host)
__device__ __forceinline__ float* xrow(const float* x, int j, int64_t ldx) {
  return reinterpret_cast<float*>(const_cast<char*>(reinterpret_cast<const char*>(x)) +
                                  uint64_t(uint32_t(j)) * uint64_t(uint32_t(ldx) * 4u));
}

// Row loads land straight in the destination registers with nothing consuming
// them here: any use (even a select) in the issuing block would make the
// compiler wait for the load on the spot.  Lanes f >= F read x[F - 1]; those
// Z entries meet zero weight rows, so they need no masking.
template <int KF>
__device__ __forceinline__ void sl_rows(const float* __restrict__ xr, int F, int lane,
                                        float (&v)[KF]) {
  // a buffer descriptor per (wave-uniform) row: 32-bit lane offsets with the
  // q * 256 B steps folded into the instruction, and the hardware range check
  // returns 0 for lanes f >= F -- no per-lane address arithmetic, no clamping
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(xr), 0, F * 4, 0x00020000);
#pragma unroll
  for (int q = 0; q < KF; ++q)
    v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 256 * q, 0));
}

// Issue the first batch of a slot (PF rows, t_i, s_j) unconditionally (empty and
// hub slots read valid rows that are ignored, so no branch joins in-flight
// loads) and park the record in the LDS ring for the aggregation.
// One piece of the issue of a slot's first batch: part 0 = logits (t_i, s_j),
// the source window and the ring record; part 1 + k = x row k.  The stream
// kernel spreads the parts over the MFMA k-steps.
template <int PART, int KF, int PFN, bool LIGHT = false>
__device__ __forceinline__ void sl_issue_part(const SlotRec& p, SlotRows<KF, PFN>& q,
                                              const float* __restrict__ x, int64_t ldx, int F,
                                              const int32_t* __restrict__ col,
                                              const float* __restrict__ st, int64_t dst_offset,
                                              SlotRing* __restrict__ ring, int lane) {
  if constexpr (PART == 0) {
    const int h = lane & 7;
    const int row = __builtin_amdgcn_readlane(p.v, 0);  // >= 0: clamped slots are real rows
    const int e0 = __builtin_amdgcn_readlane(p.v, 1);
    const int e1 = __builtin_amdgcn_readlane(p.v, 2);
    const int hw = __builtin_amdgcn_readlane(p.v, 3);
    const int jm = __builtin_amdgcn_ds_bpermute((8 + (lane >> 3)) << 2, p.v);  // message lane >> 3
    q.th = st[CHK(3, dst_offset + row, 0) * 16 + H + h];
    q.sj = st[int64_t(CHK(4, jm, 0)) * 16 + h];
    // sources of messages 8 .. 71 (one per lane), range-checked: light, hub and
    // empty slots fetch nothing
    if constexpr (!LIGHT) {  // the light path needs neither the window nor the sources
      const int nx = (p.live && hw < 0 && e1 - e0 > 8) ? e1 - e0 - 8 : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(col) + e0 + 8, 0, nx * 4, 0x00020000);
      q.cj = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
      if ((lane & 56) == 8) ring->j[lane & 7] = p.v;
    }
    if (lane == 0) ring->d = make_int4(p.live ? row : -1, e0, e1, hw);
  } else {
    constexpr int k = PART - 1;
    const int jk = __builtin_amdgcn_readlane(p.v, 8 + k);
    sl_rows<KF>(xrow(x, CHK(5, jk, 0), ldx), F, lane, q.xv[k]);
  }
}

template <int KF, int PFN>
__device__ __forceinline__ void sl_issue(const SlotRec& p, SlotRows<KF, PFN>& q,
                                         const float* __restrict__ x, int64_t ldx, int F,
                                         const int32_t* __restrict__ col,
                                         const float* __restrict__ st, int64_t dst_offset,
                                         SlotRing* __restrict__ ring, int lane) {
  sl_issue_part<0>(p, q, x, ldx, F, col, st, dst_offset, ring, lane);
  sl_issue_part<1>(p, q, x, ldx, F, col, st, dst_offset, ring, lane);
  if constexpr (PFN > 1) sl_issue_part<2>(p, q, x, ldx, F, col, st, dst_offset, ring, lane);
  if constexpr (PFN > 2) sl_issue_part<3>(p, q, x, ldx, F, col, st, dst_offset, ring, lane);
  if constexpr (PFN > 3) sl_issue_part<4>(p, q, x, ldx, F, col, st, dst_offset, ring, lane);
}

// In-register cross-lane reductions (DPP row rotate + gfx950 permlane swaps):
// a few VALU cycles each instead of a ds_bpermute round trip through the LDS
// unit per step (__shfl_xor).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float max_xor16_32(float v) {  // over lanes xor 16, 32
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
__device__ __forceinline__ float max_xor8_16_32(float v) {  // same head (lane & 7), all messages
  return max_xor16_32(fmaxf(v, dpp_mov<0x128>(v)));        // row_ror:8
}
__device__ __forceinline__ float sum_xor8_16_32(float v) {
  v += dpp_mov<0x128>(v);
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(p[0]) + __uint_as_float(p[1]);
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(q[0]) + __uint_as_float(q[1]);
}
__device__ __forceinline__ float max_wave(float v) {  // all 64 lanes
  v = fmaxf(v, dpp_mov<0x121>(v));  // row_ror:1
  v = fmaxf(v, dpp_mov<0x122>(v));  // row_ror:2
  v = fmaxf(v, dpp_mov<0x124>(v));  // row_ror:4
  return max_xor8_16_32(v);
}

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ f32x2 bcast2(float v, int l0) {  // (v@l0, v@l0+1), wave-uniform
  return f32x2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l0)),
               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l0 + 1))};
}

// x row of one message (wave-uniform source j) into lane <-> feature registers;
// ok = false fetches nothing and reads zeros (range check on an empty buffer)
template <int KF>
__device__ __forceinline__ void sl_row(const float* __restrict__ x, int64_t ldx, int F, int lane,
                                       int j, bool ok, float (&v)[KF]) {
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      xrow(x, j, ldx), 0, ok ? F * 4 : 0, 0x00020000);
#pragma unroll
  for (int q = 0; q < KF; ++q)
    v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 256 * q, 0));
}

// z += p_k x_k for rows k0 .. k0 + kn - 1 of a batch (kn >= 1; k0 a constant
// after unrolling); the weights of
// a message are broadcast as head pairs from lanes 8 k + 2 g (constant lanes).
// (Parking the weights in LDS and reading them back as two broadcast
// ds_read_b128 per message saves the 8 v_readlane but exposes the LDS latency
// in the FMA chain: measured slower with no VGPRs left to read ahead.)
template <int KF, int NR>
__device__ __forceinline__ void sl_fma(f32x2 (&z)[4][KF], const float (&xr)[NR][KF], float pv,
                                       int k0, int kn) {
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    if (k == 0 || k < kn) {
      f32x2 p2[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) p2[g] = bcast2(pv, 8 * (k0 + k) + 2 * g);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int qq = 0; qq < KF; ++qq)
          z[g][qq] = __builtin_elementwise_fma(p2[g], f32x2{xr[k][qq], xr[k][qq]}, z[g][qq]);
    }
  }
}

// Un-normalised z of one slot, heads in pairs (z2[g] = heads 2g, 2g+1, lane <->
// feature), and 1 / (sum + eps) of head lane & 7 (1 for hub rows, whose merged
// z is already normalised).  Online softmax over batches of 8 messages.
//  * batch 0: logits and rows 0..3 were issued one tile ahead (q); rows 4..7 are
//    issued on entry.
//  * batches 1..: sources come from the cj window (lane i = message cb + i,
//    loaded at issue time), so the logits and all 8 rows of the next batch are
//    issued together at the end of the current one (one memory round trip per
//    batch; a col -> st -> rows chain would be three).
template <int KF, int PFN>
__device__ __forceinline__ float sl_compute(const int4 d, const int j0, const SlotRows<KF, PFN>& q,
                                            const float* __restrict__ x, int64_t ldx, int F,
                                            int Fp, const int32_t* __restrict__ col,
                                            const float* __restrict__ st, float slope, float dp,
                                            uint64_t seed, const float* __restrict__ zhub,
                                            float* __restrict__ stats, int lane,
                                            f32x2 (&z)[4][KF]) {
  const int h = lane & 7, kk = lane >> 3;
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) z[g][qq] = f32x2{0.f, 0.f};
  if (d.x < 0) return 1.0f;
  if (d.w >= 0) {  // hub: merged row (already normalised)
    const float* src = zhub + int64_t(CHK(6, d.w, 2)) * (H * Fp);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int qq = 0; qq < KF; ++qq) {
        const int f = lane + 64 * qq;
        if (f < Fp) z[g][qq] = f32x2{src[2 * g * Fp + f], src[(2 * g + 1) * Fp + f]};
      }
    return 1.0f;
  }
  const int e0 = CHK(12, d.y, 3), e1 = CHK(13, d.z, 3);
  const int n = e1 - e0;
  float xa[4][KF], xb[4][KF];
  const float keep = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
  // batch 0
  float m, l;
  {
    const bool valid = kk < n;
    const float v = leaky01(q.sj + q.th, slope);
    m = max_xor8_16_32(valid ? v : -INFINITY);
    float pv = valid ? __expf(v - m) : 0.f;
    l = pv;
    if (dp > 0.f) pv = dropout_keep(seed, uint32_t(e0 + kk), uint32_t(h), dp) ? pv * keep : 0.f;
    sl_fma<KF, PFN>(z, q.xv, pv, 0, min(PFN, n));
#pragma unroll
    for (int k0 = PFN; k0 < 8; k0 += 4) {  // rest of the batch, 4 rows at a time
      if (n > k0) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          sl_row<KF>(x, ldx, F, lane,
                     CHK(8, __builtin_amdgcn_readlane(j0, 8 * (k0 + k < 8 ? k0 + k : 7)), 0),
                     k0 + k < n && k0 + k < 8, xb[k]);
        sl_fma<KF, 4>(z, xb, pv, k0, min(4, min(n, 8) - k0));
      }
    }
  }
  // batches 1..: loads of batch b issued at the end of batch b - 8
  int cj = q.cj, cb = 8;  // cj window: lane i = message cb + i
  float sv = 0.f;
  auto issue = [&](int b) {
    if (b - cb >= 64) {  // past the window (more than 72 messages): next 64 sources
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<int32_t*>(col) + e0 + b, 0, (n - b) * 4, 0x00020000);
      cj = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
      cb = b;
    }
    const int jl = __builtin_amdgcn_ds_bpermute((b - cb + kk) << 2, cj);
    sv = st[int64_t(CHK(7, jl, 0)) * 16 + h];
#pragma unroll
    for (int k = 0; k < 4; ++k)
      sl_row<KF>(x, ldx, F, lane, CHK(9, __builtin_amdgcn_readlane(cj, b - cb + k), 0),
                 b + k < n, xa[k]);
    if (n - b > 4) {
#pragma unroll
      for (int k = 0; k < 4; ++k)
        sl_row<KF>(x, ldx, F, lane, CHK(9, __builtin_amdgcn_readlane(cj, b - cb + 4 + k), 0),
                   b + 4 + k < n, xb[k]);
    }
  };
  if (n > 8) issue(8);
  for (int b = 8; b < n; b += 8) {
    const bool valid = b + kk < n;
    const float v = leaky01(sv + q.th, slope);
    const float bm = max_xor8_16_32(valid ? v : -INFINITY);
    const float mn = fmaxf(m, bm);
    const float sc = __expf(m - mn);
    float pv = valid ? __expf(v - mn) : 0.f;
    l = fmaf(l, sc, pv);
    if (__any(sc != 1.0f)) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x2 s2 = bcast2(sc, 2 * g);
#pragma unroll
        for (int qq = 0; qq < KF; ++qq) z[g][qq] *= s2;
      }
    }
    m = mn;
    if (dp > 0.f)
      pv = dropout_keep(seed, uint32_t(e0 + b + kk), uint32_t(h), dp) ? pv * keep : 0.f;
    sl_fma<KF, 4>(z, xa, pv, 0, min(4, n - b));
    if (n - b > 4) sl_fma<KF, 4>(z, xb, pv, 4, min(4, n - b - 4));
    if (b + 8 < n) issue(b + 8);
  }
  l = sum_xor8_16_32(l);
  if (__builtin_expect(stats != nullptr, 0) && lane < 8) {  // training only
    float* sr = stats + int64_t(CHK(11, d.x, 1)) * 16 + lane;
    sr[0] = m;
    sr[8] = l;
  }
  return __builtin_amdgcn_rcpf(l + kSoftmaxEps);
}

// lo' = f16(t - f32(hi)) for both halves of a packed pair: one v_fma_mix each
// (fp32 fma with an f16 operand, rounded to f16) instead of two conversions
// back, a subtract and a pack
__device__ __forceinline__ uint32_t split_lo(f32x2 t, uint32_t hi) {
  uint32_t lo;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lo)
      : "v"(t.x), "v"(t.y), "v"(hi));
  return lo;
}

// One slot's Z row packed for the LDS tile: normalised, power-of-two scaled
// (max |z| -> [2^13, 2^14)), feature-major (K position 8 f + h), fp16 hi and
// unscaled lo' per feature (lane + 64 q).
template <int KF>
struct SlotZ {
  f16x8 hi[KF], lo[KF];
  int er;   // row scale exponent
  int row;  // destination row (-1: empty slot)
};

// Normalise (inv of head lane & 7), scale by 2^er and split into fp16 hi / lo'
// (GS: er = erg for every row; otherwise from the row's max |z|).
template <int KF, bool GS>
__device__ __forceinline__ void sl_pack(const f32x2 (&z)[4][KF], float inv, int erg, int lane,
                                        SlotZ<KF>& o) {
  // row scale from max |z_h| * inv_h (rounding is monotonic, so this equals the
  // max of the normalised values); normalisation and scale in one multiplier
  // per head pair (inv * 2^er is exact)
  f32x2 i2[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) i2[g] = bcast2(inv, 2 * g);
  int er = erg;
  if constexpr (!GS) {
    float zm = 0.f;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      f32x2 a = {fabsf(z[g][0].x), fabsf(z[g][0].y)};
#pragma unroll
      for (int qq = 1; qq < KF; ++qq)
        a = f32x2{fmaxf(a.x, fabsf(z[g][qq].x)), fmaxf(a.y, fabsf(z[g][qq].y))};
      a *= i2[g];
      zm = fmaxf(zm, fmaxf(a.x, a.y));
    }
    zm = max_wave(zm);
    int ex = 0;
    if (zm > 0.f) frexpf(zm, &ex);
    er = 14 - ex;
    er = er > 100 ? 100 : (er < -100 ? -100 : er);
  }
  const float rs = ldexpf(1.0f, er);
  f32x2 s2[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) s2[g] = i2[g] * f32x2{rs, rs};
#pragma unroll
  for (int qq = 0; qq < KF; ++qq) {
    union { f16x8 v; f16x2 p[4]; uint32_t u[4]; } a, b;
#pragma unroll
    for (int g = 0; g < 4; ++g) {  // per head pair: pk_mul, cvt_pk, 2 fma_mix
      const f32x2 t = z[g][qq] * s2[g];
      a.p[g] = __builtin_convertvector(t, f16x2);
      b.u[g] = split_lo(t, a.u[g]);
    }
    o.hi[qq] = a.v;
    o.lo[qq] = b.v;
  }
  o.er = er;
}

// Aggregate one slot (record from the LDS ring, first batch in q) into registers.
// GS: every row takes the scale exponent erg (from max |x|, see k_stream);
// otherwise the row's own max |z| sets it.
template <int KF, int PFN, bool GS>
__device__ __forceinline__ void sl_prep(const SlotRing* __restrict__ ring, const SlotRows<KF, PFN>& q,
                                        const float* __restrict__ x, int64_t ldx, int F, int Fp,
                                        const int32_t* __restrict__ col,
                                        const float* __restrict__ st, float slope, float dp,
                                        uint64_t seed, const float* __restrict__ zhub,
                                        float* __restrict__ stats, SlotZ<KF>& o, int erg,
                                        int lane PROF_PARAMS) {
  const int4 d = uni4(ring->d);
  const int j0 = ring->j[lane >> 3];
#ifdef GFD_PROF
  const uint64_t t_in = __builtin_readcyclecounter();
#endif
  f32x2 z[4][KF];
  const float inv = sl_compute<KF, PFN>(d, j0, q, x, ldx, F, Fp, col, st, slope, dp, seed, zhub,
                                   stats, lane, z);
  PROF_MARK(9);
  sl_pack<KF, GS>(z, inv, erg, lane, o);
  o.row = d.x;
#ifdef GFD_PROF
  // slot cycles by degree class: 10/11 deg <= 4, 12/13 5..8, 14/15 > 8 (hub rows skipped)
  if (lane == 0 && d.x >= 0 && d.w < 0) {
    const int deg = d.z - d.y;
    const int c = deg <= 4 ? 10 : (deg <= 8 ? 12 : 14);
    prof_lds[(threadIdx.x >> 6) * kProfN + c] += uint32_t(__builtin_readcyclecounter() - t_in);
    prof_lds[(threadIdx.x >> 6) * kProfN + c + 1] += 1;
  }
#endif
}

// Store a prepared row into the Z tile (one 16-B write per feature and plane).
template <int KF>
__device__ __forceinline__ void sl_write(const SlotZ<KF>& o, int Fp, _Float16* __restrict__ zh,
                                         _Float16* __restrict__ zl, float* __restrict__ rsc,
                                         int* __restrict__ rid, int r, int lane) {
#pragma unroll
  for (int qq = 0; qq < KF; ++qq) {
    const int f = lane + 64 * qq;
    if (f < Fp) {
      *reinterpret_cast<f16x8*>(zh + 8 * f) = o.hi[qq];
      *reinterpret_cast<f16x8*>(zl + 8 * f) = o.lo[qq];
    }
  }
  if (lane == 0) {
    rsc[r] = ldexpf(1.0f, -o.er);
    rid[r] = o.row;
  }
}

// z = sum over the first K rows of p_k x_k (no per-message branches: rows past
// the slot's messages carry p = 0 on valid prefetched rows)
template <int KF, int K>
__device__ __forceinline__ void sl_fmaK(f32x2 (&z)[4][KF], const float (&xr)[4][KF], float pv) {
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) z[g][qq] = f32x2{0.f, 0.f};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    f32x2 p2[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) p2[g] = bcast2(pv, 8 * k + 2 * g);
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int qq = 0; qq < KF; ++qq)
        z[g][qq] = __builtin_elementwise_fma(p2[g], f32x2{xr[k][qq], xr[k][qq]}, z[g][qq]);
  }
}

// A slot with at most 4 messages (all rows prefetched), not a hub, no dropout
// -- most slots: straight-line code, the softmax sum and reciprocal independent
// of the FMA block (which has no per-message branches: rows past the slot's
// messages carry p = 0 on valid prefetched rows).  Same arithmetic as
// sl_compute + sl_pack.  kmax: messages to run (wave-uniform, >= n).
template <int KF, bool GS>
__device__ __forceinline__ void sl_light(const int4 d, const SlotRows<KF, 4>& q, int kmax,
                                         float slope, int Fp, float* __restrict__ stats,
                                         _Float16* __restrict__ zh, _Float16* __restrict__ zl,
                                         float* __restrict__ rsc, int* __restrict__ rid, int r,
                                         int erg, int lane) {
  if (d.x < 0) {  // past the last destination
    if (lane == 0) rid[r] = -1;
    return;
  }
  const int kk = lane >> 3;
  const int n = d.z - d.y;
  const float v = leaky01(q.sj + q.th, slope);
  const float m = max_xor8_16_32(kk < n ? v : -INFINITY);
  const float p = kk < n ? __expf(v - m) : 0.f;
  const float l = sum_xor8_16_32(p);
  if (__builtin_expect(stats != nullptr, 0) && lane < 8) {  // training only
    float* sr = stats + int64_t(CHK(11, d.x, 1)) * 16 + lane;
    sr[0] = m;
    sr[8] = l;
  }
  const float inv = __builtin_amdgcn_rcpf(l + kSoftmaxEps);
  f32x2 z[4][KF];
  if (kmax <= 1) sl_fmaK<KF, 1>(z, q.xv, p);
  else if (kmax == 2) sl_fmaK<KF, 2>(z, q.xv, p);
  else sl_fmaK<KF, 4>(z, q.xv, p);
  SlotZ<KF> o;
  sl_pack<KF, GS>(z, inv, erg, lane, o);
  o.row = d.x;
  sl_write<KF>(o, Fp, zh, zl, rsc, rid, r, lane);
}

template <int KF, int PFN, bool GS>
__device__ __forceinline__ void sl_store(const SlotRing* __restrict__ ring, const SlotRows<KF, PFN>& q,
                                         const float* __restrict__ x, int64_t ldx, int F, int Fp,
                                         const int32_t* __restrict__ col,
                                         const float* __restrict__ st, float slope, float dp,
                                         uint64_t seed, const float* __restrict__ zhub,
                                         float* __restrict__ stats, _Float16* __restrict__ zh,
                                         _Float16* __restrict__ zl, float* __restrict__ rsc,
                                         int* __restrict__ rid, int r, int erg,
                                         int lane PROF_PARAMS) {
  SlotZ<KF> o;
  sl_prep<KF, PFN, GS>(ring, q, x, ldx, F, Fp, col, st, slope, dp, seed, zhub, stats, o, erg,
                       lane PROF_PASS);
  sl_write<KF>(o, Fp, zh, zl, rsc, rid, r, lane);
}


// Weight-stationary streaming tile kernel (persistent, one 8-wave block per CU,
// two waves per SIMD at up to 256 VGPRs).
//
//  * The projection weights stay on chip for the launch: wave w owns column
//    tile ct = w & 3 over K half kh = w >> 2 (k-steps [kh*KH, kh*KH + KH)):
//    W_hi of its k-steps in VGPRs, W_lo of the first KH - LO in VGPRs and of
//    the last LO in LDS.  Only x rows, logits and slot records stream per tile.
//  * Z goes through LDS once per 16-row tile in the feature-major K order
//    p = 8 f + h, so a lane stores all 8 heads of its feature with one 16-B
//    write per (hi, lo).  acc += Zhi.Whi + Zhi.Wlo + Zlo.Whi (lo unscaled).
//  * Two destinations per wave (rows 2w, 2w+1).  Their first batches of x rows
//    are issued one tile ahead (in flight during the MFMA phase and the
//    reduction); their records are loaded two tiles ahead and parked in an LDS
//    ring between issue and aggregation.  After the rows are issued no load the
//    kernel waits on precedes their use (vmcnt is in order).
//  * Per tile: MFMA -> kh = 1 partials to LDS -> barrier -> kh = 0 waves reduce
//    and store out; every wave aggregates its next rows into Z -> barrier.
template <int KF, int KHM, int LO, bool EXACT, bool GS, bool LIGHT>
__global__ void __launch_bounds__(kSWaves * 64, 2) k_stream(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ wsh,
    const uint4* __restrict__ wsl, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, const float* __restrict__ zhub, float* __restrict__ out,
    float* __restrict__ stats, const float* __restrict__ xmax, int64_t num_tiles,
    const int64_t* __restrict__ split) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  const int ZS = 8 * Fp + 8;                                    // row stride (fp16), 16-B pad
  const int KH = EXACT ? KHM : Fp / 8;                          // k-steps per K half (<= KHM)
  _Float16* Zh = reinterpret_cast<_Float16*>(ssm);              // [16][ZS]
  _Float16* Zl = Zh + kTile * ZS;                               // [16][ZS]
  f32x4* red0 = reinterpret_cast<f32x4*>(Zl + kTile * ZS);      // [2 parity][4 ct][64]
  SlotRing* ring0 = reinterpret_cast<SlotRing*>(red0 + 2 * 4 * 64);  // [2 parity][16]
  float* rsc0 = reinterpret_cast<float*>(ring0 + 2 * kTile);    // [2][16] by tile parity
  int* rid0 = reinterpret_cast<int*>(rsc0 + 2 * kTile);         // [2][16]
  uint4* WL = reinterpret_cast<uint4*>(rid0 + 2 * kTile);       // [8 waves][LO][64]

  const int wave = wave_uniform(threadIdx.x >> 6);
  const int ct = wave & 3, kh = wave >> 2;
  const int r0 = 2 * wave, r1 = r0 + 1;
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  // tiles t0 + v*G, v < nv
  // LIGHT: tiles [*split, num_tiles) (every slot <= 4 messages, no hub, no
  // dropout); otherwise [0, *split)
  const int64_t tb = LIGHT ? *split : 0, te = LIGHT ? num_tiles : *split;
  const int64_t nv = t0 < te - tb ? (te - tb - 1 - t0) / G + 1 : 0;
  int lane = opaque(threadIdx.x & 63);
  auto slot = [&](int64_t v, int r) { return (tb + t0 + v * G) * kTile + r; };

  // kernel-lifetime constants first: nothing the loop waits on may be loaded
  // after the first rows are issued
  const float bcol = bias ? bias[ct * 16 + (lane & 15)] : 0.f;
  const float wu = hdr->w_unscale;
  // GS: one Z-row scale 2^erg for the launch.  Every aggregated row is a convex
  // combination of x rows (times 1 / (1 - p) under dropout), hub rows included,
  // so |z| <= max|x| * keep < 2^ex and |z| * 2^erg < 2^14 (fp16 hi and lo' normal
  // down to 2^-17 of the bound; below that the error stays < 2^-38 max|x|)
  int erg = 0;
  if constexpr (GS) {
    const float bound = *xmax * (dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f);
    int ex = 0;
    if (bound > 0.f) frexpf(bound, &ex);
    erg = 14 - ex;
    erg = __builtin_amdgcn_readfirstlane(erg > 100 ? 100 : (erg < -100 ? -100 : erg));
  }
  constexpr int NR = KHM - LO;  // k-steps (of KHM) with W_lo in registers
  f16x8 bh[KHM], bl[NR > 0 ? NR : 1];
#pragma unroll
  for (int u = 0; u < KHM; ++u) {
    uint4 vh = make_uint4(0, 0, 0, 0), vl = vh;
    if (u < KH) {
      const int idx = ((kh * KH + u) * 4 + ct) * 64 + lane;
      vh = wsh[idx];
      vl = wsl[idx];
    }
    bh[u] = *reinterpret_cast<const f16x8*>(&vh);
    if (u < NR) bl[u < NR ? u : 0] = *reinterpret_cast<const f16x8*>(&vl);
    else WL[(wave * LO + (u - NR)) * 64 + lane] = vl;
  }

#ifdef GFD_PROF
  __shared__ uint32_t prof_lds[kSWaves * kProfN];
  if (lane < kProfN) prof_lds[wave * kProfN + lane] = 0;
  uint64_t prof_t = __builtin_readcyclecounter();
#endif
  SlotRec n0, n1;
  SlotRows<KF> d0, d1;
  // prologue: tile 0 issued and aggregated; records of tile 1 loading
  sl_rec(n0, slot(0, r0), num_dst, desc, cols8, lane);
  sl_rec(n1, slot(0, r1), num_dst, desc, cols8, lane);
  sl_issue<KF, 4>(n0, d0, x, ldx, F, col, st, dst_offset, ring0 + r0, lane);
  sl_issue<KF, 4>(n1, d1, x, ldx, F, col, st, dst_offset, ring0 + r1, lane);
  sl_rec(n0, slot(1, r0), num_dst, desc, cols8, lane);
  sl_rec(n1, slot(1, r1), num_dst, desc, cols8, lane);
  if (nv > 0) {
    if constexpr (LIGHT) {
      const int4 da = uni4(ring0[r0].d), db = uni4(ring0[r1].d);
      const int kmax = max(da.z - da.y, db.z - db.y);
      sl_light<KF, GS>(da, d0, kmax, slope, Fp, stats, Zh + r0 * ZS, Zl + r0 * ZS, rsc0, rid0,
                       r0, erg, lane);
      sl_light<KF, GS>(db, d1, kmax, slope, Fp, stats, Zh + r1 * ZS, Zl + r1 * ZS, rsc0, rid0,
                       r1, erg, lane);
    } else {
      sl_store<KF, 4, GS>(ring0 + r0, d0, x, ldx, F, Fp, col, st, slope, dp, seed, zhub, stats,
                          Zh + r0 * ZS, Zl + r0 * ZS, rsc0, rid0, r0, erg, lane PROF_PASS);
      sl_store<KF, 4, GS>(ring0 + r1, d1, x, ldx, F, Fp, col, st, slope, dp, seed, zhub, stats,
                          Zh + r1 * ZS, Zl + r1 * ZS, rsc0, rid0, r1, erg, lane PROF_PASS);
    }
  }
  __syncthreads();

  // out rows of a finished tile (waves kh = 0): own K-half partial + the other
  // half's from LDS, row scale, bias
  auto reduce_store = [&](const f32x4& acc, int tpar) {
    const float* rsc = rsc0 + tpar * kTile;
    const int* rid = rid0 + tpar * kTile;
    const f32x4 sum = acc + red0[(tpar * 4 + ct) * 64 + lane];
    const int n = ct * 16 + (lane & 15);
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int r = (lane >> 4) * 4 + q;
      const int ri = rid[r];
      if (ri >= 0) out[int64_t(CHK(10, ri, 1)) * C + n] = sum[q] * (rsc[r] * wu) + bcol;
    }
  };
  f32x4 acc_prev = {0.f, 0.f, 0.f, 0.f};  // kh = 0: tile v - 1, stored during MFMA(v)
  for (int64_t v = 0; v < nv; ++v) {
    lane = opaque(threadIdx.x & 63);
    const int par = int(v & 1);
    // ---- MFMA: out[16 x 16] of column tile ct over K half kh ----
    const int aoff = (lane & 15) * ZS + 8 * (lane >> 4) + 32 * kh * KH;
    const _Float16* ah = Zh + aoff;
    const _Float16* al = Zl + aoff;
    f32x4 acc0 = {0.f, 0.f, 0.f, 0.f}, acc1 = acc0;
    // A fragments (and LDS-resident W_lo) AP k-steps ahead; the scheduling
    // barriers keep the compiler from hoisting every LDS read of the tile
    // (registers belong to W)
    constexpr int AP = LIGHT ? GFD_STREAM_AP_LIGHT : GFD_STREAM_AP;
    f16x8 phi[AP], plo[AP], pwl[AP];
#pragma unroll
    for (int u = 0; u < AP; ++u) {
      phi[u] = *reinterpret_cast<const f16x8*>(ah + 32 * u);
      plo[u] = *reinterpret_cast<const f16x8*>(al + 32 * u);
      if (u >= NR) {
        const uint4 w = WL[(wave * LO + (u - NR)) * 64 + lane];
        pwl[u] = *reinterpret_cast<const f16x8*>(&w);
      }
    }
    const int pn = par ^ 1;
    const bool more = v + 1 < nv;
#pragma unroll
    for (int u = 0; u < KHM; ++u) {
      // the next tile's first rows are issued between the k-steps: the vector
      // memory pipe is idle in this phase (issued all at once after the
      // aggregation, the 16 slots' loads queued behind each other).  Issued
      // unconditionally (past the last tile: clamped, ignored records), so no
      // copy of the previous rows has to stay live through the MFMA loop
      // the 10 issue pieces (per slot: header, 4 rows) spread evenly over the
      // k-steps: piece i in k-step i * KHM / 10
      SlotRing* rg = ring0 + pn * kTile;
#define GFD_PIECE(i) (u == (i) * KHM / 10)
      if (GFD_PIECE(0)) sl_issue_part<0, KF, 4, LIGHT>(n0, d0, x, ldx, F, col, st, dst_offset, rg + r0, lane);
      if (GFD_PIECE(1)) sl_issue_part<1, KF, 4, LIGHT>(n0, d0, x, ldx, F, col, st, dst_offset, rg + r0, lane);
      if (GFD_PIECE(2)) sl_issue_part<2, KF, 4, LIGHT>(n0, d0, x, ldx, F, col, st, dst_offset, rg + r0, lane);
      if (GFD_PIECE(3)) sl_issue_part<3, KF, 4, LIGHT>(n0, d0, x, ldx, F, col, st, dst_offset, rg + r0, lane);
      if (GFD_PIECE(4)) {
        sl_issue_part<4, KF, 4, LIGHT>(n0, d0, x, ldx, F, col, st, dst_offset, rg + r0, lane);
        sl_rec(n0, slot(v + 2, r0), num_dst, desc, cols8, lane);
      }
      if (GFD_PIECE(5)) sl_issue_part<0, KF, 4, LIGHT>(n1, d1, x, ldx, F, col, st, dst_offset, rg + r1, lane);
      if (GFD_PIECE(6)) sl_issue_part<1, KF, 4, LIGHT>(n1, d1, x, ldx, F, col, st, dst_offset, rg + r1, lane);
      if (GFD_PIECE(7)) sl_issue_part<2, KF, 4, LIGHT>(n1, d1, x, ldx, F, col, st, dst_offset, rg + r1, lane);
      if (GFD_PIECE(8)) sl_issue_part<3, KF, 4, LIGHT>(n1, d1, x, ldx, F, col, st, dst_offset, rg + r1, lane);
      if (GFD_PIECE(9)) {
        sl_issue_part<4, KF, 4, LIGHT>(n1, d1, x, ldx, F, col, st, dst_offset, rg + r1, lane);
        sl_rec(n1, slot(v + 2, r1), num_dst, desc, cols8, lane);
      }
#undef GFD_PIECE
      if (u == KHM - 2 && !kh && v > 0) reduce_store(acc_prev, pn);  // tile v - 1
      if (u < KH && kAblate != 1) {
        const f16x8 ahi = phi[u % AP], alo = plo[u % AP];
        f16x8 blo = u < NR ? bl[u < NR ? u : 0] : pwl[u % AP];
        if (u + AP < KH) {
          phi[u % AP] = *reinterpret_cast<const f16x8*>(ah + 32 * (u + AP));
          plo[u % AP] = *reinterpret_cast<const f16x8*>(al + 32 * (u + AP));
          if (u + AP >= NR) {
            const uint4 w = WL[(wave * LO + (u + AP - NR)) * 64 + lane];
            pwl[u % AP] = *reinterpret_cast<const f16x8*>(&w);
          }
        }
#ifdef GFD_MFMA_SPLITACC  // A/B: main product and corrections in separate chains
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc1, 0, 0, 0);
        acc0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bh[u], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bh[u], acc1, 0, 0, 0);
#else
        f32x4& acc = (u & 1) ? acc1 : acc0;
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, bh[u], acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(ahi, blo, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(alo, bh[u], acc, 0, 0, 0);
#endif
#ifndef GFD_NO_SCHED_BARRIER
        __builtin_amdgcn_sched_barrier(0);
#endif
      }
    }
    acc0 += acc1;
    if (kh) red0[(par * 4 + ct) * 64 + lane] = acc0;
    acc_prev = acc0;
    PROF_MARK(0);
    __syncthreads();  // partials visible; every Z read of this tile done
    PROF_MARK(1);

    // ---- tile v + 1: aggregate its rows into Z ----
    PROF_MARK(2);
    if (more && kAblate != 2) {
#ifdef GFD_PROF_WAIT  // diagnostic: time the wait for the prefetched rows separately
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      PROF_MARK(8);
#endif
      if constexpr (LIGHT) {
        const int4 da = uni4(ring0[pn * kTile + r0].d), db = uni4(ring0[pn * kTile + r1].d);
        const int kmax = max(da.z - da.y, db.z - db.y);  // wave-uniform
        sl_light<KF, GS>(da, d0, kmax, slope, Fp, stats, Zh + r0 * ZS, Zl + r0 * ZS,
                         rsc0 + pn * kTile, rid0 + pn * kTile, r0, erg, lane);
        sl_light<KF, GS>(db, d1, kmax, slope, Fp, stats, Zh + r1 * ZS, Zl + r1 * ZS,
                         rsc0 + pn * kTile, rid0 + pn * kTile, r1, erg, lane);
        PROF_MARK(19);
      } else {
        sl_store<KF, 4, GS>(ring0 + pn * kTile + r0, d0, x, ldx, F, Fp, col, st, slope, dp, seed,
                            zhub, stats, Zh + r0 * ZS, Zl + r0 * ZS, rsc0 + pn * kTile,
                            rid0 + pn * kTile, r0, erg, lane PROF_PASS);
        PROF_MARK(3);
        sl_store<KF, 4, GS>(ring0 + pn * kTile + r1, d1, x, ldx, F, Fp, col, st, slope, dp, seed,
                            zhub, stats, Zh + r1 * ZS, Zl + r1 * ZS, rsc0 + pn * kTile,
                            rid0 + pn * kTile, r1, erg, lane PROF_PASS);
        PROF_MARK(4);
      }
    }
    __syncthreads();  // Z of the next tile complete
    PROF_MARK(6);
#ifdef GFD_PROF
    if (lane == 0) prof_lds[wave * kProfN + 7] += 1;
#endif
  }
  if (nv > 0 && !kh) reduce_store(acc_prev, int((nv - 1) & 1));  // last tile
#ifdef GFD_PROF
  if (lane < kProfN) atomicAdd(&g_prof[lane], (unsigned long long)prof_lds[wave * kProfN + lane]);
#endif
}

size_t stream_smem(int Fp, int lo) {
  return sizeof(_Float16) * 2 * kTile * (8 * Fp + 8) + sizeof(f32x4) * 2 * 4 * 64 +
         sizeof(SlotRing) * 2 * kTile + sizeof(float) * 4 * kTile +
         sizeof(uint4) * kSWaves * lo * 64;
}

// ---------------------------------------------------------------------------
// Hub chunks: partial (max, sum, unnormalised z) per chunk of a heavy row.
template <int KF>
__global__ void __launch_bounds__(256) k_hub_partial(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t dst_offset, const float* __restrict__ st, float slope, float dp, uint64_t seed,
    const int4* __restrict__ chunks, int64_t num_chunks, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  if (c >= num_chunks) return;
  const int4 ck = chunks[c];
  const float t_h = st[(dst_offset + ck.w) * 16 + H + (lane & 7)];
  float acc[H][KF];
  SegState S = aggregate_segment<KF>(x, ldx, F, col, ck.y, ck.z, st, t_h, slope, dp, seed, acc);
  const int KP = H * Fp;
  float* pr = part + c * (16 + KP);
  if (lane < 8) {
    pr[lane] = S.m;
    pr[8 + lane] = S.ssum;
  }
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) {
      const int f = lane + 64 * q;
      if (f < Fp) pr[16 + hh * Fp + f] = acc[hh][q];
    }
}

// Per hub: M_h = max_c m_ch, S_h = sum_c S_ch e^(m_ch - M_h).  One wave per hub,
// lanes over chunks.  Writes hubstat[hub][16] and the backward stats.
// Hub finalisation, one wave per (hub, K slice of 256 values): global (max,
// sum) per head over the hub's chunk partials (lanes over chunks), then the
// slice of the merged, normalised z row (16-B loads, chunks unrolled by 4).
// Fp is a multiple of 8, so a 4-wide group never straddles heads.
__global__ void __launch_bounds__(256) k_hub_fin(const float* __restrict__ part, int Fp,
                                                 const int32_t* __restrict__ chunk_ptr,
                                                 const int32_t* __restrict__ hub_dst,
                                                 int64_t num_hubs, int slices,
                                                 float* __restrict__ stats,
                                                 float* __restrict__ zhub) {
  const int lane = threadIdx.x & 63;
  const int64_t wid = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t hb = wid / slices;
  const int sl = int(wid - hb * slices);
  if (hb >= num_hubs) return;
  const int KP = H * Fp;
  const int64_t stride = 16 + KP;
  const int c0 = chunk_ptr[hb], c1 = chunk_ptr[hb + 1];
  float M[H], S[H];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) { M[hh] = -INFINITY; S[hh] = 0.f; }
  for (int c = c0 + lane; c < c1; c += 64) {
    const f32x4* pr = reinterpret_cast<const f32x4*>(part + c * stride);
    const f32x4 a = pr[0], b = pr[1];
    M[0] = fmaxf(M[0], a.x); M[1] = fmaxf(M[1], a.y); M[2] = fmaxf(M[2], a.z); M[3] = fmaxf(M[3], a.w);
    M[4] = fmaxf(M[4], b.x); M[5] = fmaxf(M[5], b.y); M[6] = fmaxf(M[6], b.z); M[7] = fmaxf(M[7], b.w);
  }
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) M[hh] = fmaxf(M[hh], __shfl_xor(M[hh], o));
  for (int c = c0 + lane; c < c1; c += 64) {
    const float* pr = part + c * stride;
#pragma unroll
    for (int hh = 0; hh < H; ++hh) S[hh] += pr[8 + hh] * __expf(pr[hh] - M[hh]);
  }
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) S[hh] += __shfl_xor(S[hh], o);
  if (stats && sl == 0 && lane < H) {
    const int64_t i = hub_dst[hb];
    float m = M[0], ssum = S[0];
#pragma unroll
    for (int hh = 1; hh < H; ++hh)
      if (lane == hh) { m = M[hh]; ssum = S[hh]; }
    stats[i * 16 + lane] = m;
    stats[i * 16 + 8 + lane] = ssum;
  }
  const int k4 = sl * 64 + lane;
  if (k4 >= KP / 4) return;
  const int hh = (4 * k4) / Fp;
  float Mh = M[0], Sh = S[0];
#pragma unroll
  for (int q = 1; q < H; ++q)
    if (hh == q) { Mh = M[q]; Sh = S[q]; }
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
  for (int c = c0; c < c1; ++c) {
    const float* pr = part + c * stride;
    acc += reinterpret_cast<const f32x4*>(pr + 16)[k4] * __expf(pr[hh] - Mh);
  }
  reinterpret_cast<f32x4*>(zhub + hb * KP)[k4] = acc * (1.0f / (Sh + kSoftmaxEps));
}


// ---------------------------------------------------------------------------
inline int kf_for(int F) { return (F + 63) / 64; }

size_t fused_smem(int Fp) {  // fp16 hi + lo half-tile (= 4 B per element) + partials + rows
  return sizeof(float) * (kTile * (4 * Fp + 8) + 3 * 4 * 64 * 4 + 2 * kTile);
}

int cu_count();

gfd_status launch_logits(const float* x, int64_t rows, int F, int64_t ldx, const float* uv, int Fu,
                         float* st, float* xmax, hipStream_t stream) {
  if (rows <= 0) return GFD_OK;
  int64_t blocks = (rows + 63) / 64;  // 4 waves x 16 rows
  if (blocks > 8192) blocks = 8192;
  const uintptr_t a = reinterpret_cast<uintptr_t>(x);
  if (a % 16 == 0 && ldx % 4 == 0 && F <= 256) {
    const int64_t tiles = (rows + 15) / 16;
    int64_t nb = (tiles + 3) / 4;
    const int64_t cap = int64_t(cu_count()) * 8;  // resident blocks; grid-stride beyond
    if (nb > cap) nb = cap;
    if (F <= 176)
      k_logits_s<11><<<int(nb), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st, xmax);
    else
      k_logits_s<16><<<int(nb), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st, xmax);
    GFD_LAUNCH_CHECK();
    return GFD_OK;
  }
  if (xmax) {
    k_absmax<<<int(cu_count()) * 4, 256, 0, stream>>>(x, rows, F, ldx, xmax);
    GFD_LAUNCH_CHECK();
  }
  if (a % 16 == 0 && ldx % 4 == 0)
    k_logits<4><<<int(blocks), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st);
  else if (a % 8 == 0 && ldx % 2 == 0)
    k_logits<2><<<int(blocks), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st);
  else
    k_logits<1><<<int(blocks), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

// GFD_FUSED_MODE (profiling ablation only): 0 full, 1 aggregation only,
// 2 projection only.  Outputs are wrong in modes 1 and 2.
// Waves per SIMD the tile kernel is compiled for.  KF <= 2 fits 64 VGPRs (8 waves
// per SIMD, two blocks per CU); KF = 3 at 64 VGPRs spills ~52 B/lane per
// destination (33 GB of scratch writes at C4), so it runs at 4 waves per SIMD.
// GFD_FUSED_OCC=4|8 overrides (A/B experiments).
int fused_occ(int KF) {
  static int m = [] {
    const char* e = getenv("GFD_FUSED_OCC");
    return e ? atoi(e) : 0;
  }();
  return m ? m : (KF >= 3 ? 4 : 8);
}

int fused_mode() {
  static int m = [] {
    const char* e = getenv("GFD_FUSED_MODE");
    return e ? atoi(e) : 0;
  }();
  return m;
}

// GFD_TILE_KERNEL (A/B switch): 0 default (k_stream where its register budget
// allows, else k_fused), 1 k_fused, 2 persistent half-stationary (k_persist),
// 3 32-row tiles, 4 32-row tiles with paired aggregation.
int tile_kernel() {
  static int m = [] {
    const char* e = getenv("GFD_TILE_KERNEL");
    return e ? atoi(e) : 0;
  }();
  return m;
}

int cu_count() {
  static int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v > 0 ? v : 256;
  }();
  return n;
}

struct AggArgs {
  const float* x; int F; int64_t ldx;
  int64_t N;  // rows of x / st (checked builds only)
  const int32_t* rowptr; const int32_t* col; int64_t num_dst; int64_t dst_offset;
  const float* st; const char* packed; const float* bias; float slope; float dp; uint64_t seed;
  gfd_plan plan; int stages; float* out; float* stats;
  float* part; float* hubstat; float* zhub;
  const float* xmax;  // max |x| over all rows of x (nullable): one scale for every Z row
  int64_t* split;     // device word: first light tile (k_split / k_stream); workspace
};

constexpr size_t kLdsBytes = 160 * 1024;

size_t persist_fixed_lds(int Fp) {  // fp16 hi/lo half-tile + partials + row scale/ids
  return sizeof(_Float16) * 2 * kTile * (4 * Fp + 8) + sizeof(float) * 3 * 4 * 64 * 4 +
         sizeof(float) * 4 * kTile;
}

template <int KF>
gfd_status launch_persist(const AggArgs& a, const PackLayout& L, int64_t tiles,
                          hipStream_t stream) {
#ifdef EXP_NKW
  constexpr int NKW = EXP_NKW;
#else
  constexpr int NKW = (KF * 64 * H / 32 + 3) / 4;   // W_hi k-steps per wave (all of them)
#endif
  const size_t fixed = persist_fixed_lds(L.Fp);
  if (fixed > kLdsBytes) return GFD_ERR_UNSUPPORTED;
  int nl = int((kLdsBytes - fixed) / (sizeof(uint4) * 256));  // W_lo k-steps held in LDS
  if (nl > L.KS) nl = L.KS;
  const size_t lds = fixed + size_t(nl) * sizeof(uint4) * 256;
  static bool attr_set = false;
  if (!attr_set) {
    if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_persist<KF, NKW>),
                            hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsBytes)) !=
        hipSuccess)
      return GFD_ERR_HIP;
    attr_set = true;
  }
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  const gfd_plan& p = a.plan;
  const PackHeader* hdr = reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off);
  const uint4* whi = reinterpret_cast<const uint4*>(a.packed + L.whi_off);
  const uint4* wlo = reinterpret_cast<const uint4*>(a.packed + L.wlo_off);
  k_persist<KF, NKW><<<int(grid), kPWaves * 64, lds, stream>>>(
      a.x, a.F, L.Fp, a.ldx, a.col, a.num_dst, a.dst_offset,
      reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.st, hdr, whi, wlo, nl, a.bias,
      a.slope, a.dp, a.seed, a.zhub, a.out, a.stats, tiles);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

// First tile of the light range: tiles run in descending-degree order, so the
// slots that fit k_stream's light path (<= 4 messages, not a hub) form a
// suffix; *split = ceil(first light slot / 16) (num_tiles under dropout: the
// light path has no dropout).  One block narrows the range 1024-fold per pass.
__global__ void __launch_bounds__(1024) k_split(const int4* __restrict__ desc, int64_t num_dst,
                                                int64_t num_tiles, float dp,
                                                int64_t* __restrict__ split) {
  __shared__ int64_t s_lo, s_hi, s_first;
  const int t = threadIdx.x;
  if (dp > 0.f) {
    if (t == 0) *split = num_tiles;
    return;
  }
  auto light = [&](int64_t s) {
    if (s >= num_dst) return true;
    const int4 d = desc[s];
    return d.w < 0 && d.z - d.y <= 4;
  };
  if (t == 0) { s_lo = 0; s_hi = num_dst; }  // answer in [lo, hi]; light(num_dst) holds
  __syncthreads();
  for (;;) {
    const int64_t lo = s_lo, hi = s_hi;
    const int64_t span = hi - lo;
    const int64_t step = span <= 1024 ? 1 : (span + 1023) / 1024;
    if (t == 0) s_first = hi;
    __syncthreads();
    const int64_t p = lo + int64_t(t) * step;
    if (p < hi && light(p)) atomicMin(reinterpret_cast<unsigned long long*>(&s_first),
                                      (unsigned long long)p);
    __syncthreads();
    const int64_t f = s_first;
    if (step == 1) {
      if (t == 0) *split = (f + kTile - 1) / kTile;
      return;
    }
    __syncthreads();
    if (t == 0) {
      s_hi = f;
      s_lo = f - step + 1 > lo ? f - step + 1 : lo;
    }
    __syncthreads();
  }
}

template <int KF, int KHM, int LO, bool EXACT, bool GS>
gfd_status launch_stream_k(const AggArgs& a, const PackLayout& L, int64_t tiles,
                           hipStream_t stream) {
  auto kheavy = &k_stream<KF, KHM, LO, EXACT, GS, false>;
  auto klight = &k_stream<KF, KHM, LO, EXACT, GS, true>;
  if (EXACT && L.KS / 2 != KHM) return GFD_ERR_UNSUPPORTED;
  const size_t lds = stream_smem(L.Fp, LO);
  if (L.KS / 2 > KHM || lds > kLdsBytes || !a.plan.slot_cols || !a.split)
    return GFD_ERR_UNSUPPORTED;
  if (!(a.slope >= 0.f && a.slope <= 1.f)) return GFD_ERR_UNSUPPORTED;  // leaky01
  if (a.ldx > (int64_t(1) << 29)) return GFD_ERR_UNSUPPORTED;           // xrow: 4 ldx < 2^32
  static size_t attr_lds = 0;  // dynamic LDS the attributes currently allow
  if (lds > attr_lds) {
    for (auto kern : {kheavy, klight})
      if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                              hipFuncAttributeMaxDynamicSharedMemorySize, int(lds)) != hipSuccess)
        return GFD_ERR_HIP;
    attr_lds = lds;
  }
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  const gfd_plan& p = a.plan;
#ifdef GFD_CHECKED
  {
    const long long lim[4] = {a.N, a.num_dst, a.plan.num_hubs, 1ll << 31};
    if (hipMemcpyToSymbolAsync(HIP_SYMBOL(g_lim), lim, sizeof(lim), 0, hipMemcpyHostToDevice,
                               stream) != hipSuccess)
      return GFD_ERR_HIP;
  }
#endif
  k_split<<<1, 1024, 0, stream>>>(reinterpret_cast<const int4*>(p.slot_desc), a.num_dst, tiles,
                                  a.dp, a.split);
  GFD_LAUNCH_CHECK();
  for (auto kern : {kheavy, klight}) {  // tiles [0, split) general path, [split, tiles) light
    kern<<<int(grid), kSWaves * 64, lds, stream>>>(
        a.x, a.F, L.Fp, a.ldx, a.col, a.num_dst, a.dst_offset,
        reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.st,
        reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),
        reinterpret_cast<const uint4*>(a.packed + L.wsh_off),
        reinterpret_cast<const uint4*>(a.packed + L.wsl_off), a.bias, a.slope, a.dp, a.seed,
        a.zhub, a.out, a.stats, a.xmax, tiles, a.split);
    GFD_LAUNCH_CHECK();
  }
  return GFD_OK;
}

template <int KF, int KHM, int LO, bool EXACT>
gfd_status launch_stream_g(const AggArgs& a, const PackLayout& L, int64_t tiles,
                           hipStream_t stream) {
  return a.xmax ? launch_stream_k<KF, KHM, LO, EXACT, true>(a, L, tiles, stream)
                : launch_stream_k<KF, KHM, LO, EXACT, false>(a, L, tiles, stream);
}

// k_stream instance for this K: KH = KS / 2 k-steps per wave, at most KHM = 8 / 16 / 21
// for one / two / three feature chunks (F <= 64 / 128 / 168); GFD_ERR_UNSUPPORTED
// beyond (k_fused takes over).  KF = 3 keeps W_lo of 8 k-steps per wave in LDS.
template <int KF>
gfd_status launch_stream(const AggArgs& a, const PackLayout& L, int64_t tiles,
                         hipStream_t stream) {
  const bool exact = L.KS / 2 == (KF == 1 ? 8 : KF == 2 ? 16 : 21);
  if constexpr (KF == 1) {
    return exact ? launch_stream_g<1, 8, 0, true>(a, L, tiles, stream)
                 : launch_stream_g<1, 8, 0, false>(a, L, tiles, stream);
  } else if constexpr (KF == 2) {
    return exact ? launch_stream_g<2, 16, 0, true>(a, L, tiles, stream)
                 : launch_stream_g<2, 16, 0, false>(a, L, tiles, stream);
  } else if constexpr (KF == 3) {
    return exact ? launch_stream_g<3, 21, 8, true>(a, L, tiles, stream)
                 : launch_stream_g<3, 21, 8, false>(a, L, tiles, stream);
  }
  return GFD_ERR_UNSUPPORTED;
}

template <int KF>
gfd_status launch_aggregate(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  const int Fp = L.Fp;
  const gfd_plan& p = a.plan;
  if (p.num_hubs > 0 && (a.stages & GFD_STAGE_HUBS)) {
    int64_t blocks = (p.num_chunks + 3) / 4;
    k_hub_partial<KF><<<int(blocks), 256, 0, stream>>>(
        a.x, a.F, Fp, a.ldx, a.col, a.dst_offset, a.st, a.slope, a.dp, a.seed,
        reinterpret_cast<const int4*>(p.hub_chunk), p.num_chunks, a.part);
    GFD_LAUNCH_CHECK();
    const int slices = (L.KP / 4 + 63) / 64;
    k_hub_fin<<<unsigned((p.num_hubs * slices + 3) / 4), 256, 0, stream>>>(
        a.part, Fp, p.hub_chunk_ptr, p.hub_dst, p.num_hubs, slices, a.stats, a.zhub);
    GFD_LAUNCH_CHECK();
  }
  if (!(a.stages & GFD_STAGE_TILES)) return GFD_OK;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  if constexpr (KF <= 3) {
    if (p.slot_desc && tile_kernel() == 0) {
      gfd_status s = launch_stream<KF>(a, L, tiles, stream);
      if (s != GFD_ERR_UNSUPPORTED) return s;
    }
    if (p.slot_desc && tile_kernel() == 2) return launch_persist<KF>(a, L, tiles, stream);
    if (p.slot_desc && (tile_kernel() == 3 || tile_kernel() == 4)) {
      auto kern = tile_kernel() == 4 ? &k_pair<KF> : &k_tile32<KF>;
      const size_t lds = sizeof(_Float16) * 2 * 32 * (4 * Fp + 8) + sizeof(float) * (3 * 4 * 64 * 8 + 64);
      static bool attr_set = false;
      if (!attr_set) {
        if (hipFuncSetAttribute(reinterpret_cast<const void*>(&k_tile32<KF>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsBytes)) !=
                hipSuccess ||
            hipFuncSetAttribute(reinterpret_cast<const void*>(&k_pair<KF>),
                                hipFuncAttributeMaxDynamicSharedMemorySize, int(kLdsBytes)) !=
                hipSuccess)
          return GFD_ERR_HIP;
        attr_set = true;
      }
      const PackHeader* hdr = reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off);
      kern<<<int((a.num_dst + 31) / 32), 1024, lds, stream>>>(
          a.x, a.F, Fp, a.ldx, a.col, a.num_dst, a.dst_offset,
          reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.st, hdr,
          reinterpret_cast<const uint4*>(a.packed + L.whi_off),
          reinterpret_cast<const uint4*>(a.packed + L.wlo_off), a.bias, a.slope, a.dp, a.seed,
          a.zhub, a.out, a.stats);
      GFD_LAUNCH_CHECK();
      return GFD_OK;
    }
  }
  const PackHeader* hdr = reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off);
  const uint4* whi = reinterpret_cast<const uint4*>(a.packed + L.whi_off);
  const uint4* wlo = reinterpret_cast<const uint4*>(a.packed + L.wlo_off);
  auto kern = fused_occ(KF) == 4 ? &k_fused<KF, 4> : &k_fused<KF, 8>;
  kern<<<int(tiles), kFusedWaves * 64, fused_smem(Fp), stream>>>(
      a.x, a.F, Fp, a.ldx, a.rowptr, a.col, a.num_dst, a.dst_offset, p.row_order,
      reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.st, hdr,
      whi, wlo, a.bias, a.slope, a.dp, a.seed, p.num_hubs > 0 ? p.hub_rank : nullptr, a.zhub,
      a.out, a.stats, fused_mode());
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

bool check_hc(int heads, int channels, int F) {
  return heads == H && channels == C && F >= 1 && F <= 256;
}

gfd_status aggregate_impl(const AggArgs& a, hipStream_t stream) {
  PackLayout L = pack_layout(a.F);
  switch (kf_for(a.F)) {
    case 1: return launch_aggregate<1>(a, L, stream);
    case 2: return launch_aggregate<2>(a, L, stream);
    case 3: return launch_aggregate<3>(a, L, stream);
    case 4: return launch_aggregate<4>(a, L, stream);
    default: return GFD_ERR_UNSUPPORTED;
  }
}

gfd_status check_agg_args(const float* x, int64_t N, int F, int64_t ldx, const int32_t* rowptr,
                          const int32_t* col, int64_t num_dst, int64_t dst_offset, float dp,
                          const gfd_plan& p, float* out) {
  if (N <= 0 || num_dst < 0 || dst_offset < 0 || dst_offset + num_dst > N) return GFD_ERR_ARGUMENT;
  if (!x || !rowptr || !col || !out || ldx < F) return GFD_ERR_ARGUMENT;
  if (!(dp >= 0.f && dp < 1.f)) return GFD_ERR_ARGUMENT;
  if (p.num_hubs < 0 || p.num_chunks < 0 || p.num_hubs > 0x7fffffff) return GFD_ERR_ARGUMENT;
  if (p.num_hubs > 0 &&
      (!p.hub_rank || !p.hub_chunk || !p.hub_chunk_ptr || !p.hub_dst || p.num_chunks <= 0))
    return GFD_ERR_ARGUMENT;
  if ((num_dst + kTile - 1) / kTile > 0x7fffffff) return GFD_ERR_UNSUPPORTED;
  return GFD_OK;
}

gfd_plan plan_or_empty(const gfd_plan* p) {
  if (p) return *p;
  gfd_plan e;
  e.row_order = e.slot_desc = e.slot_cols = e.hub_rank = e.hub_chunk = e.hub_chunk_ptr = e.hub_dst = nullptr;
  e.num_hubs = e.num_chunks = 0;
  return e;
}

size_t hub_ws_layout(Carve* c, int64_t num_hubs, int64_t num_chunks, const PackLayout& L,
                     float** part, float** hubstat, float** zhub) {
  *part = c->take<float>(size_t(num_chunks) * (16 + L.KP));
  *hubstat = c->take<float>(size_t(num_hubs) * 16);
  *zhub = c->take<float>(size_t(num_hubs) * L.KP);
  return c->off;
}

}  // namespace

extern "C" {

#ifdef GFD_CHECKED
// checked builds: first bounds violation {site, value, limit, block*1000+wave}; reset after read
int gfd_debug_chk(long long* host4) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host4, HIP_SYMBOL(g_chk), sizeof(long long) * 4) != hipSuccess) return -1;
  long long z[4] = {0, 0, 0, 0};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_chk), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef GFD_PROF
// diagnostic builds: k_stream phase cycles summed over waves (see g_prof); reset after read
int gfd_debug_prof(unsigned long long* host32) {
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  if (hipMemcpyFromSymbol(host32, HIP_SYMBOL(g_prof), sizeof(unsigned long long) * kProfN) != hipSuccess)
    return -1;
  unsigned long long z[kProfN] = {};
  return hipMemcpyToSymbol(HIP_SYMBOL(g_prof), z, sizeof(z)) == hipSuccess ? 0 : -1;
}
#endif

size_t gfd_gat_packed_size(int in_features, int heads, int channels) {
  if (!check_hc(heads, channels, in_features)) return 0;
  return pack_layout(in_features).bytes;
}

gfd_status gfd_gat_pack_weights(const float* weight, const float* att_src, const float* att_dst,
                                int F, int heads, int channels, void* packed,
                                gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  if (!weight || !att_src || !att_dst || !packed) return GFD_ERR_ARGUMENT;
  PackLayout L = pack_layout(F);
  char* p = static_cast<char*>(packed);
  PackHeader* hdr = reinterpret_cast<PackHeader*>(p + L.hdr_off);
  k_wmax<<<1, 1024, 0, stream>>>(weight, H * C * F, hdr);
  GFD_LAUNCH_CHECK();
  int n_uv = 2 * H * L.Fu;
  k_pack_uv<<<(n_uv + 255) / 256, 256, 0, stream>>>(weight, att_src, att_dst, F, L.Fu,
                                                    reinterpret_cast<float*>(p + L.uv_off));
  GFD_LAUNCH_CHECK();
  int n_fr = L.KS * 4 * 64;
  k_pack_frag<<<(n_fr + 255) / 256, 256, 0, stream>>>(weight, F, L.Fp, L.KS, hdr,
                                                      reinterpret_cast<uint4*>(p + L.whi_off),
                                                      reinterpret_cast<uint4*>(p + L.wlo_off));
  GFD_LAUNCH_CHECK();
  k_pack_frag_s<<<(n_fr + 255) / 256, 256, 0, stream>>>(weight, F, L.KS, hdr,
                                                        reinterpret_cast<uint4*>(p + L.wsh_off),
                                                        reinterpret_cast<uint4*>(p + L.wsl_off));
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

gfd_status gfd_gat_logits_ex(const float* x, int64_t rows, int F, int64_t ldx,
                             const void* packed, int heads, int channels, float* st, float* xmax,
                             gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  if (rows < 0 || (rows > 0 && (!x || !packed || !st)) || ldx < F) return GFD_ERR_ARGUMENT;
  PackLayout L = pack_layout(F);
  const float* uv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + L.uv_off);
  return launch_logits(x, rows, F, ldx, uv, L.Fu, st, xmax, stream);
}

gfd_status gfd_gat_logits(const float* x, int64_t rows, int F, int64_t ldx, const void* packed,
                          int heads, int channels, float* st, gfd_stream_t stream_) {
  return gfd_gat_logits_ex(x, rows, F, ldx, packed, heads, channels, st, nullptr, stream_);
}

size_t gfd_gat_fwd_workspace_size(int64_t num_nodes, int64_t num_dst, int F, int heads,
                                  int channels, int64_t num_hubs, int64_t num_chunks) {
  if (!check_hc(heads, channels, F)) return 0;
  (void)num_dst;
  PackLayout L = pack_layout(F);
  Sizer s;
  s.take<float>(size_t(num_chunks) * (16 + L.KP));    // hub partials
  s.take<float>(size_t(num_hubs) * 16);               // per-hub (max, sum)
  s.take<float>(size_t(num_hubs) * L.KP);             // merged hub z rows
  s.take<int64_t>(1);                                 // light-tile split (tile stage)
  s.take<char>(L.bytes);                              // packed weights (gfd_gat_fwd only)
  s.take<float>(size_t(num_nodes) * 16);              // st (gfd_gat_fwd when st == NULL)
  s.take<float>(1);                                   // max |x| (gfd_gat_fwd)
  return s.off;
}

gfd_status gfd_gat_aggregate_ex(const float* x, int64_t N, int F, int64_t ldx,
                                const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                                int64_t dst_offset, const float* st, const float* xmax,
                                const void* packed, const float* bias, int heads, int channels,
                                float slope, float dp, uint64_t seed, const gfd_plan* plan,
                                int stages, float* out, float* stats, void* ws, size_t ws_bytes,
                                gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  gfd_plan p = plan_or_empty(plan);
  gfd_status s = check_agg_args(x, N, F, ldx, rowptr, col, num_dst, dst_offset, dp, p, out);
  if (s != GFD_OK) return s;
  if (!st || !packed || stages < 1 || stages > 3) return GFD_ERR_ARGUMENT;
  if (num_dst == 0) return GFD_OK;
  PackLayout L = pack_layout(F);
  AggArgs a{x, F, ldx, N, rowptr, col, num_dst, dst_offset, st, static_cast<const char*>(packed),
            bias, slope, dp, seed, p, stages, out, stats, nullptr, nullptr, nullptr, xmax,
            nullptr};
  {
    Carve c(ws, ws_bytes);
    hub_ws_layout(&c, p.num_hubs, p.num_chunks, L, &a.part, &a.hubstat, &a.zhub);
    a.split = c.take<int64_t>(1);
    if (!c.ok) {
      if (p.num_hubs > 0) return GFD_ERR_WORKSPACE;
      a.split = nullptr;  // no room for the split word: general tile path only
    }
  }
  return aggregate_impl(a, stream);
}

gfd_status gfd_gat_aggregate(const float* x, int64_t N, int F, int64_t ldx, const int32_t* rowptr,
                             const int32_t* col, int64_t num_dst, int64_t dst_offset,
                             const float* st, const void* packed, const float* bias, int heads,
                             int channels, float slope, float dp, uint64_t seed,
                             const gfd_plan* plan, int stages, float* out, float* stats, void* ws,
                             size_t ws_bytes, gfd_stream_t stream_) {
  return gfd_gat_aggregate_ex(x, N, F, ldx, rowptr, col, num_dst, dst_offset, st, nullptr, packed,
                              bias, heads, channels, slope, dp, seed, plan, stages, out, stats,
                              ws, ws_bytes, stream_);
}

gfd_status gfd_gat_fwd(const float* x, int64_t N, int F, int64_t ldx, const int32_t* rowptr,
                       const int32_t* col, const float* weight, const float* att_src,
                       const float* att_dst, const float* bias, int heads, int channels,
                       float slope, float dp, uint64_t seed, const gfd_plan* plan, float* out,
                       float* st, float* stats, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  gfd_plan p = plan_or_empty(plan);
  gfd_status s = check_agg_args(x, N, F, ldx, rowptr, col, N, 0, dp, p, out);
  if (s != GFD_OK) return s;
  if (!weight || !att_src || !att_dst) return GFD_ERR_ARGUMENT;
  if (ws_bytes < gfd_gat_fwd_workspace_size(N, N, F, heads, channels, p.num_hubs, p.num_chunks))
    return GFD_ERR_WORKSPACE;
  PackLayout L = pack_layout(F);
  Carve c(ws, ws_bytes);
  AggArgs a{x, F, ldx, N, rowptr, col, N, 0, st, nullptr, bias, slope, dp, seed, p, GFD_STAGE_ALL,
            out, stats, nullptr, nullptr, nullptr, nullptr, nullptr};
  hub_ws_layout(&c, p.num_hubs, p.num_chunks, L, &a.part, &a.hubstat, &a.zhub);
  a.split = c.take<int64_t>(1);
  void* packed = c.take<char>(L.bytes);
  float* st_ws = c.take<float>(size_t(N) * 16);
  float* xmax = c.take<float>(1);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  if (st == nullptr) st = st_ws;
  a.st = st;
  a.packed = static_cast<const char*>(packed);
  a.xmax = xmax;
  s = gfd_gat_pack_weights(weight, att_src, att_dst, F, heads, channels, packed, stream_);
  if (s != GFD_OK) return s;
  if (hipMemsetAsync(xmax, 0, sizeof(float), stream) != hipSuccess) return GFD_ERR_HIP;
  s = gfd_gat_logits_ex(x, N, F, ldx, packed, heads, channels, st, xmax, stream_);
  if (s != GFD_OK) return s;
  return aggregate_impl(a, stream);
}

}  // extern "C"
