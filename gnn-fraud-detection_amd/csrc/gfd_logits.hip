// gfd_logits.hip -- the per-node attention logits pass of PyG GATConv.forward
// (alpha_src / alpha_dst; /root/reference/src/models/gat.py:80, tgn.py:94)
// fused with the outputs of the destinations whose only message is their own
// self loop ("lone": a third of the C4 power-law graph's nodes).
//
// A lone destination's softmax has one term, alpha = 1 for every head, so
// PyG's out_i = mean_h W_h x_i + bias = Wbar x_i + bias.  The logits pass
// already streams every row of x through registers; computing Wbar x_i there
// (K = F on f16 MFMA, 3-term hi/lo split of the power-of-two scaled row,
// ~2^-21 relative) for the rows whose in-degree is 1 saves the lone kernel's
// second read of those rows.
//
// k_logits_lone: one 16-wave block per CU, grid-stride over 16-row tiles.
//   * lane (r = l & 15, g = l >> 4) loads features 16 s + 4 g .. +3 of row r
//     for every fp32 k-step s (fp32), or 32 t + 8 g .. +7 for every f16
//     k-step t (bf16) -- 16-B loads (pairs of 8-B loads for rows that are only
//     8-B aligned, e.g. a contiguous [N, 166] fp32 x), all issued before the
//     first MFMA;
//   * the row, scaled by 2^e (max |x| -> [2^13, 2^14)), is split into f16
//     hi / lo' once per f16 k-step t (fp32 k-steps 2 t and 2 t + 1 of the
//     lane, matched by the permuted fragments of k_pack_wbar_perm /
//     k_pack_uv_perm, which stay in LDS for the launch);
//   * st = x . [U | V] on v_mfma_f32_16x16x32_f16 (3-term split, ~2^-21
//     relative: 18 MFMAs per tile instead of 44 fp32 16x16x4 ones);
//   * a tile holding a row whose nonzero features span more than 2^18 (an
//     outlier feature: under one row scale the f16 split would lose the small
//     ones -- tests/test_gatconv_gpu.py::test_backward_heavy_tailed_features)
//     takes fp32 MFMA instead, with the same fragments as fp32 B operands
//     (hi + lo): exact fp32 products for its logits and lone outputs;
//   * if any row of the tile is lone: out = x . Wbar^T from the same
//     fragments (12 more MFMAs per k-step);
//   * out rows (and, in training, the softmax stats: max = leaky(s_i + t_i),
//     denominator 1) are written for lone rows only.
//   * stores: the MFMA results (lane = column, 4 rows per lane) are turned
//     row-major through a per-wave LDS scratch tile, so every lane writes 16 B
//     of one row -- the 16 rows' s | t in ONE store instruction (rows' 32-B s
//     slot and 32-B t row), a lone row's 256-B output in 16 lanes, both as
//     non-temporal stores (C4 pass 2.15 -> 1.98 ms).  The writes (1.35 GB at
//     C4) are what holds the pass above its read-only speed: without the s / t
//     stores it takes 1.72 ms, without them, the lone outputs and with
//     contiguous loads 1.18 (profiles/r5b_logits_ablation.txt).
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kLLWaves = 16;  // 1024-thread blocks, one per CU (LDS 128.5 KB)
constexpr int kTP = 68;        // scratch tile row pitch (floats): conflict-free column writes
constexpr int kLKS = 12;     // fp32 k-steps of 16 features (F <= 192)
constexpr int kLKB = 6;      // f16 k-steps of 32 features

// KS fp32 k-steps held per row (11: F <= 176, the f16 k-step 5 pairs step 10
// with zeros; 12: F <= 192).  HEAD: the model head folded into the lone rows'
// store (its own instance: the plain one stays inside 128 VGPRs, no spill)
// Order this wave's scratch-tile accesses as written (the hardware runs one
// wave's LDS operations in order; this keeps the compiler from moving them)
__device__ __forceinline__ void lds_order() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
}

template <typename XT, int KS, bool HEAD, bool A16, bool EPI>
__global__ void __launch_bounds__(kLLWaves * 64) __attribute__((amdgpu_waves_per_eu(4, 4)))
k_logits_lone(
    const typename XT::T* __restrict__ x, int64_t rows, int F, int64_t ldx,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ uph,
    const uint4* __restrict__ upl,
    const uint4* __restrict__ wph, const uint4* __restrict__ wpl,
    const int32_t* __restrict__ rowptr, const float* __restrict__ bias, float slope,
    float* __restrict__ sl, int lds, float* __restrict__ tl, int ldt, float* __restrict__ xmax,
    float* __restrict__ out,
    float* __restrict__ stats, Epi ep) {
  extern __shared__ __attribute__((aligned(16))) char lsm[];
  // permuted Wbar hi / lo fragments [2][kLKB][4][64], zero past KB
  uint4 (*WB)[kLKB][4][64] = reinterpret_cast<uint4 (*)[kLKB][4][64]>(lsm);
  // permuted [U | V] hi / lo fragments [2][kLKB][64], zero past KB
  uint4 (*UP)[kLKB][64] = reinterpret_cast<uint4 (*)[kLKB][64]>(lsm + sizeof(uint4) * 2 * kLKB * 4 * 64);
  // bias and (HEAD) head weights for the launch [2][C]
  float (*BH)[C] = reinterpret_cast<float (*)[C]>(lsm + sizeof(uint4) * 2 * kLKB * 5 * 64);
  // this wave's row-major scratch tile [16][kTP]
  float* T = reinterpret_cast<float*>(lsm + sizeof(uint4) * 2 * kLKB * 5 * 64 + sizeof(float) * 2 * C) +
             __builtin_amdgcn_readfirstlane(threadIdx.x >> 6) * (16 * kTP);
  const int KB = (F + 31) / 32;
  const int kst = (F + 15) / 16;  // fp32 k-steps incl. the ragged tail
  const int ksf = F / 16;         // fp32 k-steps fully inside the row
  for (int i = threadIdx.x; i < kLKB * 4 * 64; i += blockDim.x) {
    const bool in = i < KB * 4 * 64;
    WB[0][0][0][i] = in ? wph[i] : make_uint4(0, 0, 0, 0);
    WB[1][0][0][i] = in ? wpl[i] : make_uint4(0, 0, 0, 0);
  }
  for (int i = threadIdx.x; i < kLKB * 64; i += blockDim.x) {
    const bool in = i < KB * 64;
    UP[0][0][i] = in ? uph[i] : make_uint4(0, 0, 0, 0);
    UP[1][0][i] = in ? upl[i] : make_uint4(0, 0, 0, 0);
  }
  for (int i = threadIdx.x; i < C; i += blockDim.x) {
    BH[0][i] = bias ? bias[i] : 0.f;
    BH[1][i] = HEAD ? ep.hw[i] : 0.f;
  }
  __syncthreads();
  const int lane0 = threadIdx.x & 63;
  // 16-B row stores when every row start of the table is 16-B aligned (kernel-uniform)
  const int st_vec = __builtin_amdgcn_readfirstlane(
      (reinterpret_cast<uintptr_t>(sl) % 16 == 0) && lds % 4 == 0 &&
      (reinterpret_cast<uintptr_t>(tl) % 16 == 0) && ldt % 4 == 0);
  const int out_vec = __builtin_amdgcn_readfirstlane(
      (reinterpret_cast<uintptr_t>(out) % 16 == 0) && ep.ldo % 4 == 0);
  const float wbu = hdr->wb_unscale;
  const float uvu = hdr->uv_unscale;
  float am = 0.f;  // max |x| over the values this lane loaded
  const int64_t wave = int64_t(blockIdx.x) * kLLWaves + (threadIdx.x >> 6);
  const int64_t nwave = int64_t(gridDim.x) * kLLWaves;
  const int64_t tiles = (rows + 15) / 16;
  for (int64_t t = wave; t < tiles; t += nwave) {
    int lane = lane0, rl = lane & 15, g = lane >> 4;
    const int64_t row = t * 16 + rl;
    const bool rin = row < rows;
    // fp32: lane group g holds features 16 s + 4 g .. +3 of fp32 k-step s (the
    // permuted fragment order); bf16: features 32 t + 8 g .. +7 of f16 k-step
    // t in one 16-B load (the plain order)
    constexpr bool kH = XT::kBytes == 2;
    f32x4 a[kH ? 1 : kLKS];
    uint4 hb[kH ? kLKB : 1];
    float rm = 0.f;         // max |x| of this lane's part of the row
    float rmin = INFINITY;  // and its smallest nonzero |x|
    if constexpr (kH) {
      const uint16_t* xh = reinterpret_cast<const uint16_t*>(x) + (rin ? row : rows - 1) * ldx + 8 * g;
#pragma unroll
      for (int tt = 0; tt < kLKB; ++tt) {
        const int f0 = 32 * tt + 8 * g;
        if (tt < KB && f0 + 8 <= F) {
          if constexpr (A16) {
            hb[tt] = *reinterpret_cast<const uint4*>(xh + 32 * tt);
          } else {  // 8-B aligned rows (a row pitch of 4 k bf16): two 8-B loads
            const uint2 u0 = *reinterpret_cast<const uint2*>(xh + 32 * tt);
            const uint2 u1 = *reinterpret_cast<const uint2*>(xh + 32 * tt + 4);
            hb[tt] = make_uint4(u0.x, u0.y, u1.x, u1.y);
          }
        } else {  // ragged tail: guarded scalar loads (never past the row)
          uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
          for (int j = 0; j < 8; ++j)
            if (tt < KB && f0 + j < F) w[j >> 1] |= uint32_t(xh[32 * tt + j]) << (16 * (j & 1));
          hb[tt] = make_uint4(w[0], w[1], w[2], w[3]);
        }
      }
#pragma unroll
      for (int tt = 0; tt < kLKB; ++tt) {
        const uint32_t w[4] = {hb[tt].x, hb[tt].y, hb[tt].z, hb[tt].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v0 = fabsf(__uint_as_float(w[i] << 16));
          const float v1 = fabsf(__uint_as_float(w[i] & 0xffff0000u));
          rm = fmaxf(rm, fmaxf(v0, v1));
          rmin = fminf(rmin, fminf(v0 > 0.f ? v0 : INFINITY, v1 > 0.f ? v1 : INFINITY));
        }
      }
    } else {
      const typename XT::T* xr = x + (rin ? row : rows - 1) * ldx + 4 * g;
#pragma unroll
      for (int s = 0; s < kLKS; ++s) {
        if (s >= KS) {
          a[s] = f32x4{0.f, 0.f, 0.f, 0.f};
          continue;
        }
        if (s < ksf) {
          if constexpr (A16) {
            a[s] = load4<XT>(xr + 16 * s);
          } else {  // 8-B aligned rows (an even row pitch: the reference's [N, 166]): two 8-B loads
            const float2 u0 = *reinterpret_cast<const float2*>(xr + 16 * s);
            const float2 u1 = *reinterpret_cast<const float2*>(xr + 16 * s + 2);
            a[s] = f32x4{u0.x, u0.y, u1.x, u1.y};
          }
        } else if (s < kst) {  // ragged tail: guarded scalar loads (never past the row)
#pragma unroll
          for (int u = 0; u < 4; ++u) a[s][u] = 16 * s + 4 * g + u < F ? xcvt(xr[16 * s + u]) : 0.f;
        } else {
          a[s] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      }
#pragma unroll
      for (int s = 0; s < KS; ++s) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const float v = fabsf(a[s][u]);
          rm = fmaxf(rm, v);
          rmin = fminf(rmin, v > 0.f ? v : INFINITY);
        }
      }
    }
    const bool lone = rin && rowptr[row + 1] - rowptr[row] == 1;
    am = fmaxf(am, rm);  // clamped tail rows repeat row rows - 1: harmless for a max
    const bool any_lone = __ballot(lone) != 0;  // wave-uniform
    // Row conditioning: a row whose smallest nonzero |x| is below 2^-18 of its
    // max has features the one-row-scale f16 split cannot hold to ~2^-21 (an
    // outlier feature).  A tile with such a row also runs fp32 MFMA, and those
    // rows (only those: every other row's arithmetic stays its own, whatever
    // rows share its tile -- shards tile differently) take its results.
    const float rmax_row = max_xor16_32(rm);                 // lanes r, r + 16, r + 32, r + 48
    const float rmin_row = -max_xor16_32(-rmin);
    const bool ill = rin && rmin_row < rmax_row * 0x1p-18f;
    const bool exact = __ballot(ill) != 0;                    // wave-uniform
    const int er = scale_exp(rmax_row);
    const float rs = ldexpf(1.0f, er);
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    f32x4 o[4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) o[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
    // the lane's K value at position j (0..7) of f16 k-step tt, unscaled fp32
    // (fp32 x: the permuted order -- j < 4: fp32 k-step 2 tt, j >= 4: 2 tt + 1;
    // bf16 x: the plain order of the lane's 8-feature load)
    auto xk = [&](int tt, int j) -> float {
      if constexpr (kH) {
        const uint32_t w = (j >> 1) == 0 ? hb[tt].x : (j >> 1) == 1 ? hb[tt].y
                         : (j >> 1) == 2 ? hb[tt].z : hb[tt].w;
        return __uint_as_float((j & 1) ? (w & 0xffff0000u) : (w << 16));
      } else {
        return a[2 * tt + (j >> 2)][j & 3];
      }
    };
#pragma unroll
    for (int tt = 0; tt < kLKB; ++tt) {
      if (tt >= KB) break;  // uniform: past the row's k-steps
      union { f16x8 v; f16x2 p[4]; uint32_t u[4]; } hi, lo;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const f32x2 v = f32x2{xk(tt, 2 * i), xk(tt, 2 * i + 1)} * f32x2{rs, rs};
        hi.p[i] = __builtin_convertvector(v, f16x2);
        lo.u[i] = split_lo(v, hi.u[i]);
      }
      {
        const uint4 uh = UP[0][tt][lane], ul = UP[1][tt][lane];
        const f16x8 u_h = *reinterpret_cast<const f16x8*>(&uh);
        const f16x8 u_l = *reinterpret_cast<const f16x8*>(&ul);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi.v, u_h, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi.v, u_l, acc, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo.v, u_h, acc, 0, 0, 0);
      }
      if (any_lone) {
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) {
          const uint4 bh = WB[0][tt][ct][lane], bl = WB[1][tt][ct][lane];
          const f16x8 b_h = *reinterpret_cast<const f16x8*>(&bh);
          const f16x8 b_l = *reinterpret_cast<const f16x8*>(&bl);
          o[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi.v, b_h, o[ct], 0, 0, 0);
          o[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(hi.v, b_l, o[ct], 0, 0, 0);
          o[ct] = __builtin_amdgcn_mfma_f32_16x16x32_f16(lo.v, b_h, o[ct], 0, 0, 0);
        }
      }
    }
    float ers = ldexpf(1.0f, -er);  // the row's unscale (lanes holding row rl)
    if (exact) {
      // fp32 MFMA 16x16x4: the lane's j-th K value against the fragments'
      // j-th entry (hi + lo: the packed fp32-faithful value), 8 MFMAs per f16
      // k-step and 16-column tile; then ill rows (result element q of lane
      // (g, rl) = row 4 g + q) take these sums, unscaled
      f32x4 ae = {0.f, 0.f, 0.f, 0.f};
      f32x4 oe[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) oe[ct] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int tt = 0; tt < kLKB; ++tt) {
        if (tt >= KB) break;  // uniform: past the row's k-steps
        const uint4 uh = UP[0][tt][lane], ul = UP[1][tt][lane];
        const f16x8 u_h = *reinterpret_cast<const f16x8*>(&uh);
        const f16x8 u_l = *reinterpret_cast<const f16x8*>(&ul);
#pragma unroll
        for (int j = 0; j < 8; ++j)
          ae = __builtin_amdgcn_mfma_f32_16x16x4f32(xk(tt, j), float(u_h[j]) + float(u_l[j]), ae,
                                                   0, 0, 0);
        if (any_lone) {
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) {
            const uint4 bh = WB[0][tt][ct][lane], bl = WB[1][tt][ct][lane];
            const f16x8 b_h = *reinterpret_cast<const f16x8*>(&bh);
            const f16x8 b_l = *reinterpret_cast<const f16x8*>(&bl);
#pragma unroll
            for (int j = 0; j < 8; ++j)
              oe[ct] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                  xk(tt, j), float(b_h[j]) + float(b_l[j]), oe[ct], 0, 0, 0);
          }
        }
      }
      const int ill_i = ill ? 1 : 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        if (__builtin_amdgcn_ds_bpermute((4 * g + q) << 2, ill_i)) {
          acc[q] = ae[q];
#pragma unroll
          for (int ct = 0; ct < 4; ++ct) o[ct][q] = oe[ct][q];
        }
      }
      if (ill) ers = 1.0f;
    }
    // acc / o[ct] element q of lane l: row 4 g + q, column rl (16 ct + rl);
    // the row's unscale comes from a lane holding that row.  (Lane-derived
    // addresses below are recomputed per tile from an opaque lane id rather
    // than hoisted out of the loop and pinned in VGPRs.)
    lane = opaque(lane0);
    rl = lane & 15;
    g = lane >> 4;
    float sv[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int src = 4 * g + q;
      const float eq = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(ers)));
      sv[q] = acc[q] * (eq * uvu);
      T[src * kTP + rl] = sv[q];
    }
    lds_order();  // the wave's LDS ops run in order: no wait needed
    {  // row r = lane / 4, quarter lane % 4 (s 0..3, s 4..7, t 0..3, t 4..7)
      const int r = lane >> 2, qd = lane & 3;
      const f32x4 v = *reinterpret_cast<const f32x4*>(T + r * kTP + 4 * qd);
      const int64_t orow = t * 16 + r;
      if (orow < rows) {
        // two stores under complementary lane masks keep both table bases scalar
        auto put = [&](float* dst) {
          if (st_vec) {
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(dst));
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) dst[i] = v[i];
          }
        };
        if (qd < 2) put(sl + uint64_t(uint32_t(orow)) * uint32_t(lds) + 4 * qd);
        else put(tl + uint64_t(uint32_t(orow)) * uint32_t(ldt) + 4 * (qd - 2));
      }
    }
    const int lone_i = lone ? 1 : 0;
    if (__builtin_expect(stats != nullptr, 0) && any_lone) {  // training (no dropout) only
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int src = 4 * g + q;
        const int lq = __builtin_amdgcn_ds_bpermute(src << 2, lone_i);
        // the row's t logits (columns 8..15) next to its s logits (0..7)
        const float tq = dpp_mov<0x128>(sv[q]);  // row_ror:8 within the 16-lane row
        if (lq && rl < H) {
          const int64_t orow = t * 16 + src;
          stats[orow * 16 + rl] = leaky(sv[q] + tq, slope);
          stats[orow * 16 + H + rl] = 1.0f;
        }
      }
    }
    if (!any_lone) continue;
    if constexpr (HEAD) {  // model head: one dot per row instead of the row
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int src = 4 * g + q;  // a lane holding row src's flag and scale
        const int lq = __builtin_amdgcn_ds_bpermute(src << 2, lone_i);
        const float uq =
            __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(ers))) * wbu;
        if (lq) {  // uniform over the 16 lanes of the row (lane group g)
          const int64_t orow = t * 16 + src;
          float d = 0.f;
#pragma unroll
          for (int ct = 0; ct < 4; ++ct)
            d = fmaf(epi_store_value<EPI>(o[ct][q] * uq, BH[0][ct * 16 + rl], ct * 16 + rl, orow, ep),
                     BH[1][ct * 16 + rl], d);
          d = row16_sum(d);
          if (rl == 0) ep.hout[orow] = d + (ep.hb ? ep.hb[0] : 0.f);
        }
      }
    } else {
      // out rows through the scratch tile: lane (g, rl) writes rows 4 g + q,
      // columns 16 ct + rl; then 16 lanes x 16 B per row
      lds_order();
      int lq[4];
      float uq[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int src = 4 * g + q;
        lq[q] = __builtin_amdgcn_ds_bpermute(src << 2, lone_i);
        uq[q] = __int_as_float(__builtin_amdgcn_ds_bpermute(src << 2, __float_as_int(ers))) * wbu;
      }
      // the epilogue (its residual read) only for lone rows: other rows' slots are not stored
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) {
        const int n = ct * 16 + rl;
        const float bn = BH[0][n];
#pragma unroll
        for (int q = 0; q < 4; ++q)
          T[(4 * g + q) * kTP + n] =
              lq[q] ? epi_store_value<EPI>(o[ct][q] * uq[q], bn, n, t * 16 + 4 * g + q, ep) : 0.f;
      }
      lds_order();
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int r = 4 * i + g, ch = rl;  // row r, 16-B chunk ch of its 64 columns
        const int lr = __builtin_amdgcn_ds_bpermute(r << 2, lone_i);  // lane r holds row r's flag
        const f32x4 v = *reinterpret_cast<const f32x4*>(T + r * kTP + 4 * ch);
        if (lr) {
          float* orp = out + uint64_t(uint32_t(t * 16 + r)) * uint32_t(ep.ldo) + 4 * ch;
          if (out_vec) {
            __builtin_nontemporal_store(v, reinterpret_cast<f32x4*>(orp));
          } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) orp[k] = v[k];
          }
        }
      }
    }
  }
  if (xmax) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) am = fmaxf(am, __shfl_xor(am, o));
    if (lane0 == 0) atomic_max_nonneg(xmax, am);
  }
}

template <typename XT>
gfd_status launch_t(const void* x, int64_t rows, int F, int64_t ldx, const PackLayout& L,
                    const char* packed, const int32_t* rowptr, const float* bias, float slope,
                    float* s, int lds, float* t, int ldt, float* xmax, float* out,
                    float* stats, const Epi& ep, hipStream_t stream) {
  const int64_t tiles = (rows + 15) / 16;
  int64_t nb = (tiles + kLLWaves - 1) / kLLWaves;
  const int64_t cap = int64_t(cu_count());  // resident blocks; grid-stride beyond
  if (nb > cap) nb = cap;
  const uintptr_t xa = reinterpret_cast<uintptr_t>(x);
  const bool a16 = xa % 16 == 0 && (ldx * XT::kBytes) % 16 == 0;
  const bool k11 = F <= 176;
  // the epilogue (BN affine / ReLU / residual) and the folded head in their
  // own instances: the plain pass carries none of their code
  const bool epi = ep.ab != nullptr;
#define GFD_LL(KS, HD, A) (epi ? &k_logits_lone<XT, KS, HD, A, true> : &k_logits_lone<XT, KS, HD, A, false>)
  auto kern = a16 ? (ep.hout ? (k11 ? GFD_LL(11, true, true) : GFD_LL(12, true, true))
                             : (k11 ? GFD_LL(11, false, true) : GFD_LL(12, false, true)))
                  : (ep.hout ? (k11 ? GFD_LL(11, true, false) : GFD_LL(12, true, false))
                             : (k11 ? GFD_LL(11, false, false) : GFD_LL(12, false, false)));
#undef GFD_LL
  const size_t smem = sizeof(uint4) * 2 * kLKB * 5 * 64 + sizeof(float) * 2 * C +
                      sizeof(float) * kLLWaves * 16 * kTP;
  if (!ensure_lds(reinterpret_cast<const void*>(kern), smem)) return GFD_ERR_HIP;
  const bool plain = XT::kBytes == 2;  // bf16: plain-order fragments (16-B loads)
  kern<<<int(nb), kLLWaves * 64, smem, stream>>>(
      static_cast<const typename XT::T*>(x), rows, F, ldx,
      reinterpret_cast<const PackHeader*>(packed + L.hdr_off),
      reinterpret_cast<const uint4*>(packed + (plain ? L.ush_off : L.uph_off)),
      reinterpret_cast<const uint4*>(packed + (plain ? L.usl_off : L.upl_off)),
      reinterpret_cast<const uint4*>(packed + (plain ? L.wbh_off : L.wph_off)),
      reinterpret_cast<const uint4*>(packed + (plain ? L.wbl_off : L.wpl_off)), rowptr, bias, slope, s, lds, t, ldt,
      xmax, out, stats, ep);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

}  // namespace

namespace gfd {
namespace fwd {

bool logits_lone_supported(const void* x, int xdt, int F, int64_t ldx) {
  // fp32: 16-B loads of 4 features; bf16: 16-B loads of 8 -- or, for rows
  // only 8-B aligned (the reference's contiguous [N, 166] fp32 x), two 8-B loads
  const uintptr_t a = reinterpret_cast<uintptr_t>(x);
  const int per = xdt == GFD_DTYPE_BF16 ? 4 : 2;
  return F >= 1 && F <= 16 * kLKS && a % 8 == 0 && ldx % per == 0;
}

gfd_status launch_logits_lone(const void* x, int xdt, int64_t rows, int F, int64_t ldx,
                              const PackLayout& L, const char* packed, const int32_t* rowptr,
                              const float* bias, float slope, float* s, int lds, float* t,
                              int ldt, float* xmax, float* out, float* stats, const Epi& ep,
                              hipStream_t stream) {
  if (rows <= 0) return GFD_OK;
  if (!logits_lone_supported(x, xdt, F, ldx)) return GFD_ERR_UNSUPPORTED;
  return xdt == GFD_DTYPE_BF16
             ? launch_t<XBF16>(x, rows, F, ldx, L, packed, rowptr, bias, slope, s, lds, t, ldt,
                               xmax, out, stats, ep, stream)
             : launch_t<XF32>(x, rows, F, ldx, L, packed, rowptr, bias, slope, s, lds, t, ldt,
                              xmax, out, stats, ep, stream);
}

}  // namespace fwd
}  // namespace gfd

extern "C" {

gfd_status gfd_gat_logits_lone_split(const void* x, int x_dtype, int64_t num_nodes,
                                     int in_features, int64_t x_stride, const void* packed,
                                     int heads, int channels, const int32_t* rowptr,
                                     const float* bias, float negative_slope, float* s,
                                     int64_t s_stride, float* t, int64_t t_stride, float* xmax,
                                     float* out, int64_t out_stride, float* stats,
                                     gfd_stream_t stream_) {
  if (heads != H || channels != C || in_features < 1 || in_features > 256)
    return GFD_ERR_UNSUPPORTED;
  if (x_dtype != GFD_DTYPE_F32 && x_dtype != GFD_DTYPE_BF16) return GFD_ERR_ARGUMENT;
  if (num_nodes < 0 || x_stride < in_features) return GFD_ERR_ARGUMENT;
  if (s_stride < H || t_stride < H || s_stride > (1 << 20) || t_stride > (1 << 20) ||
      out_stride < C)
    return GFD_ERR_ARGUMENT;
  if (num_nodes > 0 && (!x || !packed || !rowptr || !s || !t || !out)) return GFD_ERR_ARGUMENT;
  const PackLayout L = pack_layout(in_features);
  return launch_logits_lone(x, x_dtype, num_nodes, in_features, x_stride, L,
                            static_cast<const char*>(packed), rowptr, bias, negative_slope, s,
                            int(s_stride), t, int(t_stride), xmax, out, stats,
                            Epi{nullptr, 0, nullptr, 0, out_stride},
                            static_cast<hipStream_t>(stream_));
}

gfd_status gfd_gat_logits_lone(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                               int64_t x_stride, const void* packed, int heads, int channels,
                               const int32_t* rowptr, const float* bias, float negative_slope,
                               float* st, float* xmax, float* out, float* stats,
                               gfd_stream_t stream_) {
  if (num_nodes > 0 && !st) return GFD_ERR_ARGUMENT;
  return gfd_gat_logits_lone_split(x, x_dtype, num_nodes, in_features, x_stride, packed, heads,
                                   channels, rowptr, bias, negative_slope, st, 16,
                                   st ? st + H : nullptr, 16, xmax, out, C, stats, stream_);
}

}  // extern "C"
