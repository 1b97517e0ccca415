// gfd_mid.hip -- general destinations (5+ messages, and the merged hub rows):
// the PyG GATConv.forward softmax-aggregate-project of
// /root/reference/src/models/gat.py:80 for the medium-degree part of a
// power-law graph, where the gather of whole x rows dominates and a single
// destination spans several batches of 8 messages.
//
// k_mid: persistent, one 16-wave block per CU (4 waves per SIMD, <= 128
// VGPRs), one destination per wave and 16-row tile.
//  * Aggregation keeps two batches (16 rows, 10.6 KB at F = 166) of every
//    wave in flight: a batch is re-issued as soon as it has been consumed, and
//    the next slot's first two batches are issued before the tile's MFMA
//    phase, so ~170 KB per CU stay in flight through it.  Sources come from
//    the slot record (first 8) and two 64-wide windows of the CSR columns
//    loaded one slot ahead; logits s_j of a batch load with its rows.
//  * Online softmax per head (running max, one rescale when it moves),
//    PyG's 1e-16 in the denominator, dropout on alpha by the counter-based
//    mask, stats for the backward.
//  * Z rows (normalised, power-of-two scaled, fp16 hi / lo') go to a 16-row
//    LDS tile in the feature-major K order p = 8 f + h; out = Z . Wcat on
//    v_mfma_f32_16x16x32_f16 (3-term split), wave (ct = w & 3, kq = w >> 2)
//    takes column tile ct over k-steps kq + 4u, W fragments stream from L2
//    (344 KB per tile at F = 166; the k_stream layout would not leave the
//    registers for 16 rows in flight), quarters summed through LDS.
//
// LDS ownership: Z rows are written after barrier 2 of the previous tile and
// read only between barriers 1 and 2; red[] is written before barrier 2 by
// kq >= 1 waves and read after it by kq = 0 waves, whose next reads of it
// follow the next barrier 2; rsc/rid are double-buffered by tile parity (the
// kq = 0 reduce of tile v reads parity v & 1 while tile v + 1 writes the other).
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kMWaves = 16;

struct MidRec {  // one slot record, one dword per lane (see sl_rec in gfd_stream.hip)
  int v;
  bool live;
};

__device__ __forceinline__ void mid_rec(MidRec& p, int64_t slot, int64_t num_dst,
                                        const int4* __restrict__ desc,
                                        const int32_t* __restrict__ cols8, int lane) {
  const int64_t sl = slot < num_dst ? slot : num_dst - 1;
  const int32_t* a = reinterpret_cast<const int32_t*>(desc + sl) + (lane & 3);
  const int32_t* b = cols8 + sl * 8 + (lane & 7);
  p.v = *((lane & 56) == 8 ? b : a);
  p.live = slot < num_dst;
}

__device__ __forceinline__ float st_at(__amdgpu_buffer_rsrc_t rs, int node, int col16);

struct MidHead {  // per-slot values loaded one slot ahead
  int4 d;         // {row (-1: empty), e_begin, e_end, hub_rank}, wave-uniform
  int j0;         // source of message lane >> 3 (first batch)
  float th;       // t_i of head lane & 7
  int cj, cjn;    // sources of messages 8 + lane and 72 + lane (0 beyond the slot)
};

// From a record: the uniform descriptor and the loads of t_i and the two
// source windows (range-checked: a short slot fetches nothing past its end).
__device__ __forceinline__ void mid_head(const MidRec& r, MidHead& h, const int32_t* __restrict__ col,
                                         __amdgpu_buffer_rsrc_t srs, int64_t dst_offset,
                                         int lane) {
  const int row = __builtin_amdgcn_readlane(r.v, 0);
  const int e0 = __builtin_amdgcn_readlane(r.v, 1);
  const int e1 = __builtin_amdgcn_readlane(r.v, 2);
  const int hw = __builtin_amdgcn_readlane(r.v, 3);
  h.d = make_int4(r.live ? row : -1, e0, e1, hw);
  h.j0 = __builtin_amdgcn_ds_bpermute((8 + (lane >> 3)) << 2, r.v);
  h.th = st_at(srs, int(dst_offset) + row, H + (lane & 7));
  const int n = (r.live && hw < 0) ? e1 - e0 : 0;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<int32_t*>(col) + e0, 0, n * 4, 0x00020000);
  h.cj = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4 + 32, 0, 0));
  h.cjn = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4 + 288, 0, 0));
}

// s_j / t_i of head h from the [N, 16] logits through a buffer descriptor
// (32-bit offsets: no 64-bit per-lane addresses to keep live)
// (node < 2^26, host-checked: the 32-bit byte offset node * 64 never wraps)
__device__ __forceinline__ float st_at(__amdgpu_buffer_rsrc_t rs, int node, int col16) {
  const uint32_t o = (uint32_t(node) * 16u + uint32_t(col16)) * 4u;
  return __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rs, int(o), 0, 0));
}

// Issue batch b (messages b .. b + 7) of a slot: the lane's logit s_j and
// the 8 rows.  w = b - w0 is the batch's offset in window cw (b >= 8), or the
// first batch comes from the record (b == 0).
template <typename XT, int KF>
__device__ __forceinline__ void mid_issue(int b, int n, int w, int cw, int j0,
                                          const void* __restrict__ x, int64_t ldx, int F,
                                          __amdgpu_buffer_rsrc_t srs, int lane, float& s,
                                          float (&X)[8][KF]) {
  const int kk = lane >> 3;
  const int js = b == 0 ? j0 : __builtin_amdgcn_ds_bpermute((w + kk) << 2, cw);
  s = st_at(srs, js, lane & 7);
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int jk = b == 0 ? __builtin_amdgcn_readlane(j0, 8 * k)
                          : __builtin_amdgcn_readlane(cw, w + k);
    row_regs<XT, KF>(xrow<XT>(x, jk, ldx), F, lane, b + k < n, X[k]);
  }
}

// z += p_k x_k over the rows k < kn of a batch with scalar FMAs: the weight
// of (message k, head h) is an SGPR broadcast (v_readlane), the row value the
// VGPR operand -- no packed-pair copies of the rows.
template <int KF>
__device__ __forceinline__ void fma_rows_s(f32x2 (&z)[4][KF], const float (&xr)[8][KF], float pv,
                                           int kn) {
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    if (k == 0 || k < kn) {
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float p0 = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), 8 * k + 2 * g));
        const float p1 =
            __int_as_float(__builtin_amdgcn_readlane(__float_as_int(pv), 8 * k + 2 * g + 1));
#pragma unroll
        for (int qq = 0; qq < KF; ++qq) {
          z[g][qq].x = fmaf(p0, xr[k][qq], z[g][qq].x);
          z[g][qq].y = fmaf(p1, xr[k][qq], z[g][qq].y);
        }
      }
    }
  }
}

template <typename XT, int KF>
__global__ void __launch_bounds__(kMWaves * 64) k_mid(
    const void* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    int64_t num_dst, int64_t dst_offset, const int4* __restrict__ desc,
    const int32_t* __restrict__ cols8, const float* __restrict__ st,
    const PackHeader* __restrict__ hdr, const uint4* __restrict__ wsh,
    const uint4* __restrict__ wsl, const float* __restrict__ bias, float slope, float dp,
    uint64_t seed, const float* __restrict__ zhub, float* __restrict__ out,
    float* __restrict__ stats, const float* __restrict__ xmax,
    const int64_t* __restrict__ split) {
  extern __shared__ __attribute__((aligned(16))) char msm[];
  const int ZS = 8 * Fp + 8;                                  // row stride (fp16), 16-B pad
  _Float16* Zh = reinterpret_cast<_Float16*>(msm);            // [16][ZS]
  _Float16* Zl = Zh + kTile * ZS;                             // [16][ZS]
  f32x4* red = reinterpret_cast<f32x4*>(Zl + kTile * ZS);     // [3 kq][4 ct][64]
  float* rsc0 = reinterpret_cast<float*>(red + 3 * 4 * 64);   // [2][16] by tile parity
  int* rid0 = reinterpret_cast<int*>(rsc0 + 2 * kTile);       // [2][16]

  const int wave = wave_uniform(threadIdx.x >> 6);
  const int ct = wave & 3, kq = wave >> 2;
  const int64_t G = gridDim.x;
  const int64_t t0 = blockIdx.x;
  const int64_t te = split ? (split[0] + kTile - 1) / kTile : (num_dst + kTile - 1) / kTile;
  const int64_t nv = t0 < te ? (te - 1 - t0) / G + 1 : 0;
  if (nv == 0) return;  // uniform per block
  int lane = opaque(threadIdx.x & 63);
  auto slot = [&](int64_t v) { return (t0 + v * G) * kTile + wave; };

  const float keep = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
  const int erg = global_scale_exp(xmax, dp);
  const float wu = hdr->w_unscale;
  const float bcol = bias ? bias[ct * 16 + (lane & 15)] : 0.f;
  const int KS = Fp / 4;  // k-steps over K = 8 Fp
  const __amdgpu_buffer_rsrc_t srs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(st), 0, int(0xffffffffu), 0x00020000);
  const __amdgpu_buffer_rsrc_t whs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(wsh), 0, KS * 4 * 64 * 16, 0x00020000);
  const __amdgpu_buffer_rsrc_t wls = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint4*>(wsl), 0, KS * 4 * 64 * 16, 0x00020000);
  auto wfrag = [&](__amdgpu_buffer_rsrc_t rs, int s) {
    const int o = ((s * 4 + ct) * 64 + lane) * 16;
    uint4 r;
    r.x = __builtin_amdgcn_raw_buffer_load_b32(rs, o, 0, 0);
    r.y = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 4, 0, 0);
    r.z = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 8, 0, 0);
    r.w = __builtin_amdgcn_raw_buffer_load_b32(rs, o + 12, 0, 0);
    return r;
  };

  MidRec rn, rnn;    // records of slots v + 1 and v + 2
  MidHead hc, hn;    // heads of slots v and v + 1
  float sA, sB;
  float XA[8][KF], XB[8][KF];
  mid_rec(rn, slot(0), num_dst, desc, cols8, lane);
  mid_head(rn, hc, col, srs, dst_offset, lane);
  mid_rec(rn, slot(1), num_dst, desc, cols8, lane);
  {  // first two batches of slot 0
    const int n = hc.d.x >= 0 && hc.d.w < 0 ? hc.d.z - hc.d.y : 0;
    mid_issue<XT, KF>(0, n, 0, 0, hc.j0, x, ldx, F, srs, lane, sA, XA);
    mid_issue<XT, KF>(8, n, 0, hc.cj, hc.j0, x, ldx, F, srs, lane, sB, XB);
  }

  for (int64_t v = 0; v < nv; ++v) {
    lane = opaque(threadIdx.x & 63);
    const int par = int(v & 1);
    // next slot's head (its windows arrive during this slot's aggregation) and
    // the record after it
    mid_head(rn, hn, col, srs, dst_offset, lane);
    mid_rec(rnn, slot(v + 2), num_dst, desc, cols8, lane);

    // ---- aggregate slot v ----
    const int4 d = hc.d;
    f32x2 z[4][KF];
#pragma unroll
    for (int g = 0; g < 4; ++g)
#pragma unroll
      for (int qq = 0; qq < KF; ++qq) z[g][qq] = f32x2{0.f, 0.f};
    float inv = 1.0f;
    if (d.x >= 0 && d.w >= 0) {  // hub: merged, normalised row (k_hub_fin)
      const float* src = zhub + int64_t(d.w) * (H * Fp);
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int qq = 0; qq < KF; ++qq) {
          const int f = lane + 64 * qq;
          if (f < Fp) z[g][qq] = f32x2{src[2 * g * Fp + f], src[(2 * g + 1) * Fp + f]};
        }
    } else if (d.x >= 0) {
      const int n = d.z - d.y, e0 = d.y;
      const int h = lane & 7, kk = lane >> 3;
      float m = -INFINITY, l = 0.f;
      int w0 = 8, cw = hc.cj, cwn = hc.cjn;  // window cw holds messages w0 .. w0 + 63
      auto consume = [&](int b, float s, const float (&X)[8][KF]) {
        const bool valid = b + kk < n;
        const float vv = leaky01(s + hc.th, slope);
        const float mn = fmaxf(m, max_xor8_16_32(valid ? vv : -INFINITY));
        const float sc = __expf(m - mn);  // 0 on the first batch, 1 while the max holds
        float p = valid ? __expf(vv - mn) : 0.f;
        l = fmaf(l, sc, p);
        if (b > 0 && __any(sc != 1.0f)) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const f32x2 s2 = bcast2(sc, 2 * g);
#pragma unroll
            for (int qq = 0; qq < KF; ++qq) z[g][qq] *= s2;
          }
        }
        m = mn;
        if (dp > 0.f)
          p = dropout_keep(seed, uint32_t(e0 + b + kk), uint32_t(h), dp) ? p * keep : 0.f;
        fma_rows_s<KF>(z, X, p, min(8, n - b));
      };
      // window of batch b (b >= 8); moves on when b leaves the current window
      auto window = [&](int b) {
        if (b - w0 >= 64) {
          cw = cwn;
          w0 += 64;
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              const_cast<int32_t*>(col) + e0 + w0 + 64, 0, max(n - w0 - 64, 0) * 4, 0x00020000);
          cwn = int(__builtin_amdgcn_raw_buffer_load_b32(rs, lane * 4, 0, 0));
        }
      };
      // two batches in flight; a consumed buffer is re-issued unconditionally
      // (batches past the slot fetch nothing: range check), so the buffers
      // keep their registers through the loop
      for (int b = 0;; b += 16) {
        consume(b, sA, XA);
        window(b + 16);
        mid_issue<XT, KF>(b + 16, n, b + 16 - w0, cw, 0, x, ldx, F, srs, lane, sA, XA);
        if (b + 8 >= n) break;
        consume(b + 8, sB, XB);
        window(b + 24);
        mid_issue<XT, KF>(b + 24, n, b + 24 - w0, cw, 0, x, ldx, F, srs, lane, sB, XB);
        if (b + 16 >= n) break;
      }
      l = sum_xor8_16_32(l);
      if (__builtin_expect(stats != nullptr, 0) && lane < 8) {  // training only
        float* sr = stats + int64_t(d.x) * 16 + lane;
        sr[0] = m;
        sr[8] = l;
      }
      inv = __builtin_amdgcn_rcpf(l + kSoftmaxEps);
    }
    {
      f16x8 zhi[KF], zlo[KF];
      const int er = pack_zrow<KF>(z, inv, erg, zhi, zlo);
      write_zrow<KF>(zhi, zlo, Fp, lane, Zh + wave * ZS, Zl + wave * ZS);
      if (lane == 0) {
        rsc0[par * kTile + wave] = ldexpf(1.0f, -er);
        rid0[par * kTile + wave] = d.x;
      }
    }

    // ---- W fragments of this wave's first k-steps (ahead of the rows in the
    // in-order vmcnt queue), then the next slot's first two batches: in
    // flight through the MFMA phase ----
    constexpr int UQ = KF == 1 ? 4 : (KF == 2 ? 8 : 11);  // k-steps per quarter (KS <= 4 UQ)
    constexpr int PD = 3;                                 // B-fragment prefetch depth
    uint4 bq[PD][2];
#pragma unroll
    for (int p = 0; p < PD; ++p) {
      const int s = kq + 4 * p;
      bq[p][0] = bq[p][1] = make_uint4(0, 0, 0, 0);
      if (s < KS) {
        bq[p][0] = wfrag(whs, s);
        bq[p][1] = wfrag(wls, s);
      }
    }
    hc = hn;
    rn = rnn;
    {
      const int n = hc.d.x >= 0 && hc.d.w < 0 ? hc.d.z - hc.d.y : 0;
      mid_issue<XT, KF>(0, n, 0, 0, hc.j0, x, ldx, F, srs, lane, sA, XA);
      mid_issue<XT, KF>(8, n, 0, hc.cj, hc.j0, x, ldx, F, srs, lane, sB, XB);
    }
    __syncthreads();  // Z tile complete

    // ---- out[16 x 16] of column tile ct over k-steps kq + 4u ----
    {
      const _Float16* ah = Zh + (lane & 15) * ZS + 8 * (lane >> 4);
      const _Float16* al = Zl + (lane & 15) * ZS + 8 * (lane >> 4);
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int u = 0; u < UQ; ++u) {
        const int s = kq + 4 * u;
        if (s < KS) {
          const f16x8 a_h = *reinterpret_cast<const f16x8*>(ah + 32 * s);
          const f16x8 a_l = *reinterpret_cast<const f16x8*>(al + 32 * s);
          const f16x8 b_h = *reinterpret_cast<const f16x8*>(&bq[u % PD][0]);
          const f16x8 b_l = *reinterpret_cast<const f16x8*>(&bq[u % PD][1]);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_h, b_h, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_h, b_l, acc, 0, 0, 0);
          acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a_l, b_h, acc, 0, 0, 0);
          const int sn = s + 4 * PD;
          if (u + PD < UQ && sn < KS) {
            bq[u % PD][0] = wfrag(whs, sn);
            bq[u % PD][1] = wfrag(wls, sn);
          }
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (kq) red[((kq - 1) * 4 + ct) * 64 + lane] = acc;
      __syncthreads();  // partials visible; every Z read of this tile done
      if (!kq) {
        acc += red[(0 * 4 + ct) * 64 + lane] + red[(1 * 4 + ct) * 64 + lane] +
               red[(2 * 4 + ct) * 64 + lane];
        const float* rsc = rsc0 + par * kTile;
        const int* rid = rid0 + par * kTile;
        const int nc = ct * 16 + (lane & 15);
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int r = (lane >> 4) * 4 + q;
          const int ri = rid[r];
          if (ri >= 0) out[int64_t(ri) * C + nc] = acc[q] * (rsc[r] * wu) + bcol;
        }
      }
    }
  }
}

size_t mid_smem(int Fp) {
  return sizeof(_Float16) * 2 * kTile * (8 * Fp + 8) + sizeof(f32x4) * 3 * 4 * 64 +
         sizeof(float) * 4 * kTile;
}

template <typename XT, int KF>
gfd_status launch_mid_k(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  auto kern = &k_mid<XT, KF>;
  const size_t lds = mid_smem(L.Fp);
  if (lds > kLdsBytes) return GFD_ERR_UNSUPPORTED;
  if (!ensure_lds(reinterpret_cast<const void*>(kern), lds)) return GFD_ERR_HIP;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  int64_t grid = cu_count();
  if (grid > tiles) grid = tiles;
  const gfd_plan& p = a.plan;
  // without light/lone classes (dropout, or no class split) every tile is general
  const int64_t* split = a.dp > 0.f ? nullptr : p.class_split;
  kern<<<int(grid), kMWaves * 64, lds, stream>>>(
      a.x, a.F, L.Fp, a.ldx, a.col, a.num_dst, a.dst_offset,
      reinterpret_cast<const int4*>(p.slot_desc), p.slot_cols, a.st,
      reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),
      reinterpret_cast<const uint4*>(a.packed + L.wsh_off),
      reinterpret_cast<const uint4*>(a.packed + L.wsl_off), a.bias, a.slope, a.dp, a.seed,
      a.zhub, a.out, a.stats, a.xmax, split);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

template <typename XT>
gfd_status launch_mid_x(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  switch (kf_for(a.F)) {
    case 1: return launch_mid_k<XT, 1>(a, L, stream);
    case 2: return launch_mid_k<XT, 2>(a, L, stream);
    case 3: return launch_mid_k<XT, 3>(a, L, stream);
    default: return GFD_ERR_UNSUPPORTED;
  }
}

}  // namespace

namespace gfd {
namespace fwd {

gfd_status launch_mid(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  const gfd_plan& p = a.plan;
  if (!p.slot_desc || !p.slot_cols) return GFD_ERR_UNSUPPORTED;
  if (a.N >= (int64_t(1) << 26)) return GFD_ERR_UNSUPPORTED;  // st byte offsets in 32 bits
  if (!(a.slope >= 0.f && a.slope <= 1.f)) return GFD_ERR_UNSUPPORTED;  // leaky01
  return a.xdt == GFD_DTYPE_BF16 ? launch_mid_x<XBF16>(a, L, stream)
                                 : launch_mid_x<XF32>(a, L, stream);
}

}  // namespace fwd
}  // namespace gfd
