// gfd_fused.hip -- general-purpose fused tile kernel (PyG GATConv.forward,
// concat=False; /root/reference/src/models/gat.py:80): used for F > 168 (four
// feature chunks, outside k_stream's register budget) and for plans
// without slot descriptors.  16 destinations per block, one per wave.
//   phase A  online softmax over the destination's CSR segment, x rows
//            gathered once for all 8 heads (lane <-> feature), z in registers
//   phase B  out = Z . Wcat + bias on f16 MFMA 16x16x32, two head-halves
//            through a 43 KB LDS tile; 3-term split hi.hi + (hi.lo + lo.hi)/2^11
//            on power-of-two-scaled rows (~2^-21 relative, fp32-faithful)
// W fragments stream from L2 per tile (344 KB at F = 166), which is why the
// plan-driven kernels replace it wherever their layouts fit.
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kFusedWaves = 16;  // one destination per wave

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

template <typename XT, int KF, int OCC>
__global__ void __launch_bounds__(1024, OCC) k_fused(
    const void* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, int64_t num_dst,
    const int32_t* __restrict__ order, const int4* __restrict__ desc,
    const float* __restrict__ s, int lds, const float* __restrict__ t, int ldt,
    const PackHeader* __restrict__ hdr,
    const uint4* __restrict__ whi, const uint4* __restrict__ wlo, const float* __restrict__ bias,
    float slope, float dp, uint64_t seed, const int32_t* __restrict__ hub_rank,
    const float* __restrict__ zhub, float* __restrict__ out, float* __restrict__ stats,
    Epi ep) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int KH4 = 4 * Fp;                 // K of one head-half
  const int ZS = KH4 + 8;                 // padded row stride (fp16 elements, 16 B pad)
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
  if (slot < num_dst) {
    if (desc) {
      dsc = desc[slot];
    } else {
      const int32_t r = order ? order[slot] : int32_t(slot);
      dsc = make_int4(r, rowptr[r], rowptr[r + 1], hub_rank ? hub_rank[r] : -1);
    }
    i = dsc.x;
  }
  if (i >= 0) {
    const int hr = hub_rank ? dsc.w : -1;
    if (hr >= 0) {  // merged (normalised) by k_hub_fin
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
      const float t_h = lrow(t, int(i), ldt)[lane & 7];
      SegState S = aggregate_segment<XT, KF>(x, ldx, F, col, e0, e1, s, lds, t_h, slope, dp, seed, z);
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
  // power-of-two row scale: max |z| -> [2^13, 2^14)
  float zm = 0.f;
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int q = 0; q < KF; ++q) zm = fmaxf(zm, fabsf(z[hh][q]));
  const int er = scale_exp(max_wave(zm));
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
      if (ri >= 0) out[int64_t(ri) * ep.ldo + n] = epi_store_value(accv[q] * (rscale[r] * wu), b, n, ri, ep);
    }
  }
}

size_t fused_smem(int Fp) {  // fp16 hi + lo half-tile (= 4 B per element) + partials + rows
  return sizeof(float) * (kTile * (4 * Fp + 8) + 3 * 4 * 64 * 4 + 2 * kTile);
}

// KF = 1 fits 64 VGPRs (8 waves per SIMD, two blocks per CU); KF >= 2 (two
// batches of rows in flight in aggregate_segment) runs at 4 waves per SIMD.
template <typename XT, int KF>
gfd_status launch_fused_t(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  const gfd_plan& p = a.plan;
  const int64_t tiles = (a.num_dst + kTile - 1) / kTile;
  auto kern = KF >= 2 ? &k_fused<XT, KF, 4> : &k_fused<XT, KF, 8>;
  kern<<<int(tiles), kFusedWaves * 64, fused_smem(L.Fp), stream>>>(
      a.x, a.F, L.Fp, a.ldx, a.rowptr, a.col, a.num_dst, p.row_order,
      reinterpret_cast<const int4*>(p.slot_desc), a.s, a.lds, a.t, a.ldt,
      reinterpret_cast<const PackHeader*>(a.packed + L.hdr_off),
      reinterpret_cast<const uint4*>(a.packed + L.whi_off),
      reinterpret_cast<const uint4*>(a.packed + L.wlo_off), a.bias, a.slope, a.dp, a.seed,
      p.num_hubs > 0 ? p.hub_rank : nullptr, a.zhub, a.out, a.stats, a.ep);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

template <typename XT>
gfd_status launch_fused_x(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  switch (kf_for(a.F)) {
    case 1: return launch_fused_t<XT, 1>(a, L, stream);
    case 2: return launch_fused_t<XT, 2>(a, L, stream);
    case 3: return launch_fused_t<XT, 3>(a, L, stream);
    case 4: return launch_fused_t<XT, 4>(a, L, stream);
    default: return GFD_ERR_UNSUPPORTED;
  }
}

}  // namespace

namespace gfd {
namespace fwd {

gfd_status launch_fused(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  if (a.ep.hout) return GFD_ERR_UNSUPPORTED;  // the model head is folded by the tile kernels
  if (a.num_dst <= 0) return GFD_OK;
  if ((a.num_dst + kTile - 1) / kTile > 0x7fffffff) return GFD_ERR_UNSUPPORTED;
  return a.xdt == GFD_DTYPE_BF16 ? launch_fused_x<XBF16>(a, L, stream)
                                 : launch_fused_x<XF32>(a, L, stream);
}

}  // namespace fwd
}  // namespace gfd
