// gfd_fwd.h -- shared pieces of the GATConv forward kernels (gfx950).
//
// The forward (PyG GATConv.forward, concat=False; called at
// /root/reference/src/models/gat.py:80 and tgn.py:94) runs aggregate-then-project:
//   z_ih = sum_j alpha_ijh x_j   (gathered x rows, F wide, fp32 accumulation)
//   out_i = sum_h W_h z_ih / H + bias   (MFMA over K = 8 * Fp)
// Destinations are scheduled by class (the plan's descending-degree slot order):
//   hubs  (> threshold messages)   k_hub_partial / k_hub_fin   (gfd_hub.hip)
//   general (hub rows, 7+ msgs)    k_stream<LIGHT = false>  8 waves, W stationary
//   light (2..kLightMax = 6 msgs)  k_stream<LIGHT = true>   (gfd_stream.hip)
//   lone  (self loop only)         k_lone   out = mean_h W_h x_i  (gfd_lone.hip)
//   F > 168 / no plan              k_fused  (gfd_fused.hip)
#pragma once

#include <type_traits>

#include "gfd_common.h"

namespace gfd {
namespace fwd {

constexpr int H = kHeads;
constexpr int C = kChannels;
constexpr int kTile = 16;             // destinations per MFMA tile (M of 16x16x32)
constexpr float kLoScale = 2048.f;    // 2^11: k_fused's re-normalised lo parts
constexpr size_t kLdsBytes = 160 * 1024;

typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef _Float16 f16x2 __attribute__((ext_vector_type(2)));
typedef float f32x2 __attribute__((ext_vector_type(2)));

// ---------------------------------------------------------------------------
// Packed weights (gfd_gat_pack_weights).
struct PackLayout {
  int F, Fp, Fu, KP, KS, KB;
  size_t hdr_off, uv_off, whi_off, wlo_off, wsh_off, wsl_off, wbh_off, wbl_off, wph_off, wpl_off,
      uph_off, upl_off, ush_off, usl_off, bytes;
};

inline PackLayout pack_layout(int F) {
  PackLayout L;
  L.F = F;
  L.Fp = (F + 7) / 8 * 8;     // K per head; 4*Fp (a head-half) is a multiple of 32
  L.Fu = (F + 15) / 16 * 16;  // logit-vector row stride
  L.KP = H * L.Fp;
  L.KS = L.KP / 32;           // MFMA k-steps over all heads
  L.KB = (F + 31) / 32;       // k-steps of the head-mean matrix (k_lone)
  size_t o = 0;
  L.hdr_off = o; o = align_up(o + 64, 256);
  L.uv_off = o; o = align_up(o + sizeof(float) * 2 * H * L.Fu, 256);
  // head-major fragments (k_fused): K position p = h * Fp + f, lo scaled by 2^11
  L.whi_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.wlo_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  // feature-major fragments (k_stream): K position p = 8 f + h, lo unscaled
  L.wsh_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.wsl_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  // head-mean matrix Wbar = mean_h W_h (k_lone): K position p = f, lo unscaled
  L.wbh_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 4 * 64, 256);
  L.wbl_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 4 * 64, 256);
  // the same matrix in the logits pass's lane order (k_logits_lone): in k-step t
  // lane group g holds features 32 t + 4 g .. +3 and 32 t + 16 + 4 g .. +3
  L.wph_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 4 * 64, 256);
  L.wpl_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 4 * 64, 256);
  // the 2H logit vectors [U | V] as f16 hi / lo B fragments (one 16-column
  // tile) in the same lane order (k_logits_lone's logits on f16 MFMA)
  L.uph_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 64, 256);
  L.upl_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 64, 256);
  // ... and in the plain order (lane group g of k-step t: features 32 t + 8 g
  // .. +7, the bf16 logits pass's 16-B loads)
  L.ush_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 64, 256);
  L.usl_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KB) * 64, 256);
  L.bytes = o;
  return L;
}

struct PackHeader {    // device-side, written by k_wmax (uv_*: k_pack_uv_perm)
  float w_unscale;     // 2^-kw   (W / H fragments scaled by 2^kw)
  float w_scale;       // 2^kw
  float wb_unscale;    // 2^-kb   (Wbar fragments scaled by 2^kb)
  float wb_scale;      // 2^kb
  float uv_unscale;    // 2^-ku   ([U | V] fragments scaled by 2^ku)
  float uv_scale;      // 2^ku
};

// ---------------------------------------------------------------------------
// Feature element types.  x is fp32 (configs C1-C4) or bf16 (config C5);
// every kernel converts on load and accumulates in fp32.
struct XF32 {
  typedef float T;
  static constexpr int kBytes = 4;
};
struct XBF16 {
  typedef uint16_t T;
  static constexpr int kBytes = 2;
};

__device__ __forceinline__ float xcvt(float v) { return v; }
__device__ __forceinline__ float xcvt(uint16_t v) { return __uint_as_float(uint32_t(v) << 16); }

// Four consecutive features of one row as fp32 (16-B fp32 / 8-B bf16 load).
template <typename XT>
__device__ __forceinline__ f32x4 load4(const typename XT::T* p) {
  if constexpr (XT::kBytes == 4) {
    return *reinterpret_cast<const f32x4*>(p);
  } else {
    const uint2 u = *reinterpret_cast<const uint2*>(p);
    return f32x4{__uint_as_float(u.x << 16), __uint_as_float(u.x & 0xffff0000u),
                 __uint_as_float(u.y << 16), __uint_as_float(u.y & 0xffff0000u)};
  }
}

// x row j as a byte pointer: an unsigned 32 x 32 -> 64-bit product (two scalar
// multiplies instead of a sign-extended 64-bit one); j >= 0 and the row pitch
// in bytes < 2^32 (checked on the host)
template <typename XT>
__device__ __forceinline__ const char* xrow(const void* x, int j, int64_t ldx) {
  return reinterpret_cast<const char*>(x) +
         uint64_t(uint32_t(j)) * uint64_t(uint32_t(ldx) * uint32_t(XT::kBytes));
}

// One gathered row in lane <-> feature layout: v[q] = x[j][lane + 64 q] for
// f < F, 0 beyond (hardware range check on a per-row buffer descriptor; the
// q step sits in the VGPR offset, which the range check covers).  ok = false
// fetches nothing and reads zeros.  Loads land straight in the registers; no
// instruction here consumes them.
template <typename XT, int KF>
__device__ __forceinline__ void row_regs(const char* xr, int F, int lane, bool ok, float (&v)[KF]) {
  // ok is wave-uniform at every call; readfirstlane keeps the descriptor
  // scalar when the compiler cannot prove it (else: a waterfall loop per load)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char*>(xr), 0, __builtin_amdgcn_readfirstlane(ok ? F * XT::kBytes : 0),
      0x00020000);
#pragma unroll
  for (int q = 0; q < KF; ++q) {
    if constexpr (XT::kBytes == 4) {
      v[q] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4 + 256 * q, 0, 0));
    } else {
      const uint32_t b = __builtin_amdgcn_raw_buffer_load_b16(rs, lane * 2 + 128 * q, 0, 0);
      v[q] = __uint_as_float(b << 16);
    }
  }
}

// Lane layouts of a gathered row held in registers by the tile kernels.
//  RowL<XT, KF, false>: KF registers, register q = feature lane + 64 q (row_regs).
//  RowL<XBF16, 3, true>: bf16 rows with 128 < F <= 192 whose starts are 4-B
//    aligned: 2 registers -- the raw bf16 pair of features 2 lane, 2 lane + 1
//    (one 4-B load) and feature 128 + lane (one 2-B load) -- so a row costs 2
//    VGPRs instead of 3.  Aggregation chunk q is then feature feat(q, lane).
// x(v, q): the fp32 value of chunk q of a held row.
template <typename XT, int KF, bool PR>
struct RowL {
  static constexpr int W = KF;
  __device__ static __forceinline__ int feat(int q, int lane) { return lane + 64 * q; }
  __device__ static __forceinline__ void load(const char* xr, int F, int lane, bool ok,
                                              float (&v)[W]) {
    row_regs<XT, KF>(xr, F, lane, ok, v);
  }
  __device__ static __forceinline__ float x(const float (&v)[W], int q) { return v[q]; }
};
template <>
struct RowL<XBF16, 3, true> {
  static constexpr int W = 2;
  __device__ static __forceinline__ int feat(int q, int lane) {
    return q < 2 ? 2 * lane + q : 128 + lane;
  }
  __device__ static __forceinline__ void load(const char* xr, int F, int lane, bool ok,
                                              float (&v)[W]) {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char*>(xr), 0, __builtin_amdgcn_readfirstlane(ok ? F * 2 : 0), 0x00020000);
    v[0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
    v[1] = __uint_as_float(uint32_t(__builtin_amdgcn_raw_buffer_load_b16(rs, 256 + lane * 2, 0, 0))
                           << 16);
  }
  __device__ static __forceinline__ float x(const float (&v)[W], int q) {
    return q == 0 ? __uint_as_float(__float_as_uint(v[0]) << 16)
         : q == 1 ? __uint_as_float(__float_as_uint(v[0]) & 0xffff0000u) : v[1];
  }
};

// ---------------------------------------------------------------------------
// Cross-lane helpers: DPP row rotates + gfx950 permlane swaps (a few VALU
// cycles each instead of a ds_bpermute round trip per step).
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float max_xor16_32(float v) {
  auto p = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = fmaxf(__uint_as_float(p[0]), __uint_as_float(p[1]));
  auto q = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return fmaxf(__uint_as_float(q[0]), __uint_as_float(q[1]));
}
// over lanes of the same head (lane & 7): all 8 messages of a batch
__device__ __forceinline__ float max_xor8_16_32(float v) {
  return max_xor16_32(fmaxf(v, dpp_mov<0x128>(v)));  // row_ror:8
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

__device__ __forceinline__ f32x2 bcast2(float v, int l0) {  // (v@l0, v@l0+1), wave-uniform
  return f32x2{__int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l0)),
               __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), l0 + 1))};
}

__device__ __forceinline__ int4 uni4(int4 v) {
  return make_int4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                   __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}

// An opaque copy: addresses derived from it are recomputed where used instead
// of being hoisted out of a persistent loop and pinned in VGPRs.
__device__ __forceinline__ int opaque(int v) {
  asm volatile("" : "+v"(v));
  return v;
}

// lo' = f16(t - f32(hi)) for both halves of a packed pair: one v_fma_mix each
__device__ __forceinline__ uint32_t split_lo(f32x2 t, uint32_t hi) {
  uint32_t lo;
  asm("v_fma_mixlo_f16 %0, %1, 1.0, -%3 op_sel_hi:[0,0,1]\n\t"
      "v_fma_mixhi_f16 %0, %2, 1.0, -%3 op_sel:[0,0,1] op_sel_hi:[0,0,1]"
      : "=&v"(lo)
      : "v"(t.x), "v"(t.y), "v"(hi));
  return lo;
}

// Row scale exponent: max |z| -> [2^13, 2^14) so fp16 hi and lo' stay normal.
__device__ __forceinline__ int scale_exp(float zmax) {
  int ex = 0;
  if (zmax > 0.f) frexpf(zmax, &ex);
  int er = 14 - ex;
  return er > 100 ? 100 : (er < -100 ? -100 : er);
}

// One-scale-per-launch exponent from max |x| (every aggregated row is a convex
// combination of x rows, times 1/(1-p) under dropout).  Returns 127 when the
// bound is too large for one scale to keep small rows accurate (max |x| >
// 2^20: rows 2^-25 of the bound would lose the lo term) -- the kernels then
// take each row's own max |z| instead.
__device__ __forceinline__ int global_scale_exp(const float* xmax, float dp) {
  if (!xmax) return 127;
  const float bound = *xmax * (dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f);
  if (!(bound <= 1048576.f)) return 127;  // also NaN / inf
  return __builtin_amdgcn_readfirstlane(scale_exp(bound));
}

// Normalise (inv of head lane & 7), scale by 2^er and split one destination's
// z (head pairs, lane <-> feature) into fp16 hi / lo' feature-major rows (K
// position 8 f + h).  erg < 127: that exponent for every row; otherwise from
// the row's own max |z|.  Returns the exponent used.
template <int KF>
__device__ __forceinline__ int pack_zrow(const f32x2 (&z)[4][KF], float inv, int erg,
                                         f16x8 (&hi)[KF], f16x8 (&lo)[KF]) {
  f32x2 i2[4];
#pragma unroll
  for (int g = 0; g < 4; ++g) i2[g] = bcast2(inv, 2 * g);
  int er = erg;
  if (erg == 127) {
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
    er = scale_exp(max_wave(zm));
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
    hi[qq] = a.v;
    lo[qq] = b.v;
  }
  return er;
}

// Split an already normalised and scaled z row into fp16 hi / lo'.
template <int KF>
__device__ __forceinline__ void split_zrow(const f32x2 (&z)[4][KF], f16x8 (&hi)[KF],
                                           f16x8 (&lo)[KF]) {
#pragma unroll
  for (int qq = 0; qq < KF; ++qq) {
    union { f16x8 v; f16x2 p[4]; uint32_t u[4]; } a, b;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      a.p[g] = __builtin_convertvector(z[g][qq], f16x2);
      b.u[g] = split_lo(z[g][qq], a.u[g]);
    }
    hi[qq] = a.v;
    lo[qq] = b.v;
  }
}

// Store a packed row into a Z tile (one 16-B write per feature and plane).
template <int KF, typename RL = RowL<XF32, KF, false>>
__device__ __forceinline__ void write_zrow(const f16x8 (&hi)[KF], const f16x8 (&lo)[KF], int Fp,
                                           int lane, _Float16* __restrict__ zh,
                                           _Float16* __restrict__ zl) {
#pragma unroll
  for (int qq = 0; qq < KF; ++qq) {
    const int f = RL::feat(qq, lane);
    if (f < Fp) {
      *reinterpret_cast<f16x8*>(zh + 8 * f) = hi[qq];
      *reinterpret_cast<f16x8*>(zl + 8 * f) = lo[qq];
    }
  }
}

// z += p_k x_k for rows k < kn of a batch (k0 a constant after unrolling); the
// weights of a message are broadcast as head pairs from lanes 8 k + 2 g.
template <int KF, int NR, typename RL = RowL<XF32, KF, false>>
__device__ __forceinline__ void fma_rows(f32x2 (&z)[4][KF], const float (&xr)[NR][RL::W],
                                         float pv, int k0, int kn) {
#pragma unroll
  for (int k = 0; k < NR; ++k) {
    if (k == 0 || k < kn) {
      f32x2 p2[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) p2[g] = bcast2(pv, 8 * (k0 + k) + 2 * g);
#pragma unroll
      for (int qq = 0; qq < KF; ++qq) {
        const float xq = RL::x(xr[k], qq);
#pragma unroll
        for (int g = 0; g < 4; ++g)
          z[g][qq] = __builtin_elementwise_fma(p2[g], f32x2{xq, xq}, z[g][qq]);
      }
    }
  }
}

// z = sum over the first K rows of p_k x_k (no per-message branches: rows past
// the slot's messages carry p = 0 on valid prefetched rows)
template <int KF, int K, int NR, typename RL = RowL<XF32, KF, false>>
__device__ __forceinline__ void fma_k(f32x2 (&z)[4][KF], const float (&xr)[NR][RL::W], float pv) {
  static_assert(K <= NR, "rows past the prefetched ones");
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
    for (int qq = 0; qq < KF; ++qq) {
      const float xq = RL::x(xr[k], qq);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        z[g][qq] = __builtin_elementwise_fma(p2[g], f32x2{xq, xq}, z[g][qq]);
    }
  }
}

// fma_k with the message weights from LDS: ab[8 k + h] = p of message k, head
// h (the wave wrote its 64 lanes' p there); two broadcast 16-B reads per
// message give the four head pairs as VGPR pairs -- 2 LDS reads instead of 8
// v_readlane per message.
template <int KF, int K, int NR, typename RL = RowL<XF32, KF, false>>
__device__ __forceinline__ void fma_k_lds(f32x2 (&z)[4][KF], const float (&xr)[NR][RL::W],
                                          const float* __restrict__ ab) {
  static_assert(K <= NR, "rows past the prefetched ones");
#pragma unroll
  for (int g = 0; g < 4; ++g)
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) z[g][qq] = f32x2{0.f, 0.f};
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const f32x4 a0 = *reinterpret_cast<const f32x4*>(ab + 8 * k);
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(ab + 8 * k + 4);
    const f32x2 p2[4] = {f32x2{a0.x, a0.y}, f32x2{a0.z, a0.w}, f32x2{a1.x, a1.y},
                         f32x2{a1.z, a1.w}};
#pragma unroll
    for (int qq = 0; qq < KF; ++qq) {
      const float xq = RL::x(xr[k], qq);
#pragma unroll
      for (int g = 0; g < 4; ++g)
        z[g][qq] = __builtin_elementwise_fma(p2[g], f32x2{xq, xq}, z[g][qq]);
    }
    // (keeps the compiler from hoisting every read of the slot: the register
    // budget has no room for them)
    __builtin_amdgcn_sched_barrier(0);
  }
}

// One destination segment (or hub chunk) on one wave, single pass with an
// online softmax.  Logit lane layout: lane = 8 k + h (message k of a batch of
// 8, head h); aggregation lane layout: lane <-> feature f = lane + 64 q.
// Returns the running max (head lane & 7) and the denominator; acc[h][q] =
// sum_j p_jh x_j[f] relative to that max.  (Measured at C4: the hub chunks
// run at ~5 TB/s with one batch in flight per wave at 5 waves per SIMD;
// keeping a second batch in flight cost occupancy and time.)
struct SegState {
  float m;
  float ssum;
};

// Logits rows: the source logits s live in [N, lds] (columns 0..H-1, global
// node rows), the destination logits t in [num_dst, ldt] (local destination
// rows).  [N, 16] st tables are s = st, t = st + 16 dst_offset + H, both
// strides 16; the sharded exchange gathers s as [N, 8] rows.  One unsigned
// 32 x 32 -> 64-bit product per row (v_mad_u64_u32), as xrow.
__device__ __forceinline__ const float* lrow(const float* p, int r, int ld) {
  return p + uint64_t(uint32_t(r)) * uint64_t(uint32_t(ld));
}

template <typename XT, int KF>
__device__ __forceinline__ SegState aggregate_segment(const void* __restrict__ x, int64_t ldx,
                                                      int F, const int32_t* __restrict__ col,
                                                      int e0, int e1, const float* __restrict__ s,
                                                      int lds, float t_h, float slope, float dp,
                                                      uint64_t seed, float (&acc)[H][KF]) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  const float keep_scale = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) acc[hh][q] = 0.f;
  float m = -INFINITY, l = 0.f;
  // sources through 64-wide windows of col (lane i = message wb + i), the
  // next window loaded one window ahead, so a batch's logits and rows are one
  // memory round trip; and batch b + 8 is issued before batch b is consumed
  // (two batches of rows in flight per wave).  Clamped: every load is in
  // bounds; the issue past the last batch fetches rows of message e1 - 1.
  int wb = e0;
  int cw = col[min(e0 + lane, e1 - 1)];
  int cn = col[min(e0 + 64 + lane, e1 - 1)];
  auto issue = [&](int b, float& sv, float (&xv)[8][KF]) {
    if (b - wb == 64) {
      wb = b;
      cw = cn;
      cn = col[min(b + 64 + lane, e1 - 1)];
    }
    const int j = __builtin_amdgcn_ds_bpermute((b - wb + kk) << 2, cw);
    sv = lrow(s, j, lds)[h];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      // plain loads, f >= F reads x[F - 1] and selects 0: never the row padding
      const typename XT::T* xr = reinterpret_cast<const typename XT::T*>(
          xrow<XT>(x, __builtin_amdgcn_readlane(cw, b - wb + k), ldx));
#pragma unroll
      for (int q = 0; q < KF; ++q) {
        const int f = lane + 64 * q;
        const float t = xcvt(xr[f < F ? f : F - 1]);
        xv[k][q] = f < F ? t : 0.f;
      }
    }
  };
  // batch b: online softmax step and the 8 rows' FMAs
  auto consume = [&](int b, float sv, const float (&xv)[8][KF]) {
    const int e = b + kk;
    const bool valid = e < e1;
    const float v = leaky(sv + t_h, slope);
    const float mn = fmaxf(m, max_xor8_16_32(valid ? v : -INFINITY));
    const float sc = __expf(m - mn);  // 0 on the first batch, 1 while the max holds
    float p = valid ? __expf(v - mn) : 0.f;
    l = fmaf(l, sc, p);
    if (b != e0 && __any(sc != 1.0f)) {  // wave-uniform: rescale the running sums
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), hh));
#pragma unroll
        for (int q = 0; q < KF; ++q) acc[hh][q] *= r;
      }
    }
    m = mn;
    if (dp > 0.f) p = dropout_keep(seed, uint32_t(e), uint32_t(h), dp) ? p * keep_scale : 0.f;
    const int nk = min(8, e1 - b);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < nk) {
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
          // p of a padding message is 0 (its clamped row is a valid one)
          const float pk =
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 8 * k + hh));
#pragma unroll
          for (int q = 0; q < KF; ++q) acc[hh][q] = fmaf(pk, xv[k][q], acc[hh][q]);
        }
      }
    }
  };
  float sv, xv[8][KF];
  issue(e0, sv, xv);
  for (int b = e0; b < e1; b += 8) {
    float sn, xn[8][KF];
    issue(b + 8, sn, xn);
    consume(b, sv, xv);
    sv = sn;
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int q = 0; q < KF; ++q) xv[k][q] = xn[k][q];
  }
  return {m, sum_xor8_16_32(l)};
}

// aggregate_segment for bf16 rows with 128 < F <= 192 whose rows start 4-B
// aligned: lane l holds features 2 l, 2 l + 1 (one 4-B load: a bf16 pair) and
// 128 + l (one 2-B load), so a row takes 2 VGPRs instead of 3 and NBF batches
// of 8 rows fit in flight at 4 waves per SIMD (C5's hub chunks: half the bytes
// of an fp32 row per message, so twice the rows in flight for the same bytes
// per round trip).  acc[h][0 / 1] = features 2 l / 2 l + 1, acc[h][2] =
// feature 128 + l (seg_feat).  Arithmetic identical to aggregate_segment.
__device__ __forceinline__ int seg_feat_pair(int q, int lane) {
  return q < 2 ? 2 * lane + q : 128 + lane;
}
template <int NBF>
__device__ __forceinline__ SegState aggregate_segment_bf16p(
    const void* __restrict__ x, int64_t ldx, int F, const int32_t* __restrict__ col, int e0,
    int e1, const float* __restrict__ s, int lds, float t_h, float slope, float dp, uint64_t seed,
    float (&acc)[H][3]) {
  static_assert(NBF >= 2 && NBF <= 4, "2 .. 4 batches in flight");
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  const float keep_scale = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < 3; ++q) acc[hh][q] = 0.f;
  float m = -INFINITY, l = 0.f;
  int wb = e0;
  int cw = col[min(e0 + lane, e1 - 1)];
  int cn = col[min(e0 + 64 + lane, e1 - 1)];
  const int f2 = 128 + lane < F ? 128 + lane : F - 1;  // clamped: never the row padding
  const bool v2 = 128 + lane < F;
  auto issue = [&](int b, float& sv, uint32_t (&xp)[8], uint32_t (&xs)[8]) {
    if (b - wb == 64) {
      wb = b;
      cw = cn;
      cn = col[min(b + 64 + lane, e1 - 1)];
    }
    const int j = __builtin_amdgcn_ds_bpermute((b - wb + kk) << 2, cw);
    sv = lrow(s, j, lds)[h];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const uint16_t* xr = reinterpret_cast<const uint16_t*>(
          xrow<XBF16>(x, __builtin_amdgcn_readlane(cw, b - wb + k), ldx));
      xp[k] = *reinterpret_cast<const uint32_t*>(xr + 2 * lane);
      xs[k] = xr[f2];
    }
  };
  auto consume = [&](int b, float sv, const uint32_t (&xp)[8], const uint32_t (&xs)[8]) {
    const int e = b + kk;
    const bool valid = e < e1;
    const float v = leaky(sv + t_h, slope);
    const float mn = fmaxf(m, max_xor8_16_32(valid ? v : -INFINITY));
    const float sc = __expf(m - mn);
    float p = valid ? __expf(v - mn) : 0.f;
    l = fmaf(l, sc, p);
    if (b != e0 && __any(sc != 1.0f)) {
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        const float r = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(sc), hh));
#pragma unroll
        for (int q = 0; q < 3; ++q) acc[hh][q] *= r;
      }
    }
    m = mn;
    if (dp > 0.f) p = dropout_keep(seed, uint32_t(e), uint32_t(h), dp) ? p * keep_scale : 0.f;
    const int nk = min(8, e1 - b);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < nk) {
        const float x0 = __uint_as_float(xp[k] << 16);
        const float x1 = __uint_as_float(xp[k] & 0xffff0000u);
        const float x2 = v2 ? __uint_as_float(xs[k] << 16) : 0.f;
#pragma unroll
        for (int hh = 0; hh < H; ++hh) {
          const float pk =
              __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 8 * k + hh));
          acc[hh][0] = fmaf(pk, x0, acc[hh][0]);
          acc[hh][1] = fmaf(pk, x1, acc[hh][1]);
          acc[hh][2] = fmaf(pk, x2, acc[hh][2]);
        }
      }
    }
  };
  float sv[NBF];
  uint32_t xp[NBF][8], xs[NBF][8];
#pragma unroll
  for (int u = 0; u < NBF - 1; ++u) issue(e0 + 8 * u, sv[u], xp[u], xs[u]);
  for (int b = e0; b < e1; b += 8 * NBF) {
#pragma unroll
    for (int u = 0; u < NBF; ++u) {
      const int bb = b + 8 * u;
      if (bb >= e1) break;  // wave-uniform
      const int w = (u + NBF - 1) % NBF;
      issue(bb + 8 * (NBF - 1), sv[w], xp[w], xs[w]);
      consume(bb, sv[u], xp[u], xs[u]);
    }
  }
  return {m, sum_xor8_16_32(l)};
}

// ---------------------------------------------------------------------------
// Host side.
// Output epilogue of the reference layer body (gat.py:82-91, eval mode), applied
// where the GATConv output row is stored: y = conv + bias, then
//   y = y * a[n] + b[n]  (BatchNorm1d with running stats folded to an affine)
//   y = max(y, 0)        (relu)
//   y += res[row, n]     (residual: the layer input, same rows as out)
// ab == NULL: plain GATConv output.  ab = [a[0..63] | b[0..63]].
struct Epi {
  const float* ab;
  int relu;
  const float* res;
  int64_t ldr;
  int64_t ldo = C;  // output row stride (floats): out row i at out + i * ldo
  // the model head Linear(C, 1) (gat.py:94) folded into the store: hout[i] =
  // y_i . hw + hb[0] is written INSTEAD of the row (hout == NULL: no head)
  const float* hw = nullptr;
  const float* hb = nullptr;
  float* hout = nullptr;
};

// Sum over the 16 lanes of a DPP row (lanes 16 k .. 16 k + 15): every lane
// of the row ends with the row's sum (the head's dot over 16 columns).
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x124, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x122, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x121, 0xF, 0xF, false));
  return v;
}

// EPI = false: an instance without the epilogue (e.ab == NULL at run time).
template <bool EPI = true>
__device__ __forceinline__ float epi_store_value(float v, float bias_n, int n, int64_t row,
                                                 const Epi& e) {
  float y = v + bias_n;
  if constexpr (!EPI) return y;
  if (e.ab) {
    y = fmaf(y, e.ab[n], e.ab[C + n]);
    if (e.relu) y = fmaxf(y, 0.f);
    if (e.res) y += e.res[row * e.ldr + n];
  }
  return y;
}

struct AggArgs {
  const void* x; int xdt; int F; int64_t ldx;
  int64_t N;
  const int32_t* rowptr; const int32_t* col; int64_t num_dst; int64_t dst_offset;
  const float* s; int lds;  // source logits [N, lds] (lrow)
  const float* t; int ldt;  // destination logits [num_dst, ldt], local rows
  const char* packed; const float* bias; float slope; float dp; uint64_t seed;
  gfd_plan plan; int stages; float* out; float* stats;
  float* part; float* zhub;
  const float* xmax;  // max |x| over all rows of x (nullable): one scale for every Z row
  Epi ep;             // output epilogue (ep.ab == NULL: none)
};

int cu_count();
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel, size)
bool ensure_lds(const void* kernel, size_t bytes);

gfd_status launch_hubs(const AggArgs& a, const PackLayout& L, hipStream_t stream);
// tile stages; GFD_ERR_UNSUPPORTED when the configuration is outside the kernel's set
gfd_status launch_general(const AggArgs& a, const PackLayout& L, hipStream_t stream);
gfd_status launch_light(const AggArgs& a, const PackLayout& L, bool to_end, hipStream_t stream);
gfd_status launch_lone(const AggArgs& a, const PackLayout& L, hipStream_t stream);
gfd_status launch_fused(const AggArgs& a, const PackLayout& L, hipStream_t stream);
gfd_status launch_logits(const void* x, int xdt, int64_t rows, int F, int64_t ldx,
                         const float* uv, int Fu, float* st, float* xmax, hipStream_t stream);
// logits fused with the lone destinations' outputs (gfd_logits.hip)
bool logits_lone_supported(const void* x, int xdt, int F, int64_t ldx);
gfd_status launch_logits_lone(const void* x, int xdt, int64_t rows, int F, int64_t ldx,
                              const PackLayout& L, const char* packed, const int32_t* rowptr,
                              const float* bias, float slope, float* s, int lds, float* t,
                              int ldt, float* xmax, float* out, float* stats, const Epi& ep,
                              hipStream_t stream);

inline int kf_for(int F) { return (F + 63) / 64; }

}  // namespace fwd
}  // namespace gfd
