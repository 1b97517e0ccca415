// gfd_pack.hip -- weight packing and per-node attention logits (the projection
// and alpha_src / alpha_dst steps of PyG GATConv.forward; reference call site
// /root/reference/src/models/gat.py:80, tgn.py:94).
//
//   k_pack_stage1 block 0: power-of-two scales for W / H and for Wbar =
//                 mean_h W_h (dev_wmax); other blocks: folded logit vectors
//                 U_h = W_h^T a_src[h], V_h = W_h^T a_dst[h] (dev_pack_uv)
//   k_pack_stage2 fp16 hi / lo MFMA B-fragments (head-major, feature-major,
//                 Wbar in two lane orders) and the [U | V] fragments, by block range
//   k_logits_s    st[n] = (x_n . U_h, x_n . V_h) on fp32 MFMA (exact fp32 chains),
//                 plus max |x| for the tile stage's one-scale-per-launch Z rows
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

// One block: max |W| / H and max |Wbar| -> the two power-of-two scales.
__device__ __forceinline__ void dev_wmax(const float* __restrict__ W, int F,
                                         PackHeader* __restrict__ hdr) {
  __shared__ float red[2][1024];
  const int t = threadIdx.x;
  const int n = H * C * F;
  float m0 = 0.f, m1 = 0.f;
  // (latency-bound on one block: 16-B loads, eight in flight per thread)
  if (reinterpret_cast<uintptr_t>(W) % 16 == 0) {
    const f32x4* W4 = reinterpret_cast<const f32x4*>(W);
    const int n4 = n / 4;  // n = 512 F: a multiple of 4
#pragma unroll 8
    for (int i = t; i < n4; i += 1024) {
      const f32x4 v = W4[i];
      m0 = fmaxf(m0, fmaxf(fmaxf(fabsf(v.x), fabsf(v.y)), fmaxf(fabsf(v.z), fabsf(v.w))));
    }
  } else {
#pragma unroll 8
    for (int i = t; i < n; i += 1024) m0 = fmaxf(m0, fabsf(W[i]));
  }
#pragma unroll 2
  for (int i = t; i < C * F; i += 1024) {  // Wbar[c][f] = mean_h W[h C + c][f]
    float s = 0.f;
#pragma unroll
    for (int h = 0; h < H; ++h) s += W[size_t(h) * C * F + i];
    m1 = fmaxf(m1, fabsf(s * (1.0f / H)));
  }
  red[0][t] = m0;
  red[1][t] = m1;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (t < s) {
      red[0][t] = fmaxf(red[0][t], red[0][t + s]);
      red[1][t] = fmaxf(red[1][t], red[1][t + s]);
    }
    __syncthreads();
  }
  if (t == 0) {
    const int kw = scale_exp(red[0][0] * (1.0f / H));  // packed values are W / H
    const int kb = scale_exp(red[1][0]);
    hdr->w_scale = ldexpf(1.0f, kw);
    hdr->w_unscale = ldexpf(1.0f, -kw);
    hdr->wb_scale = ldexpf(1.0f, kb);
    hdr->wb_unscale = ldexpf(1.0f, -kb);
  }
}

__device__ __forceinline__ void dev_pack_uv(const float* __restrict__ W,
                                            const float* __restrict__ as,
                                            const float* __restrict__ ad, int F, int Fu,
                                            float* __restrict__ uv, int bid) {
  int idx = bid * 1024 + threadIdx.x;
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

// Head-major fragments (k_fused): K position p = h Fp + f; lo' = (v - hi) 2^11.
__device__ __forceinline__ void dev_pack_frag(int bid, const float* __restrict__ W, int F, int Fp, int KS,
                            const PackHeader* __restrict__ hdr, uint4* __restrict__ whi,
                            uint4* __restrict__ wlo) {
  int idx = bid * 256 + threadIdx.x;  // (s, ct, lane)
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

// Feature-major fragments (k_stream): K position p = 8 f + h (one 16-B Z
// store per feature holds all 8 heads), lo = v - hi unscaled (|lo| <= 2^3 for
// the 2^14-scaled W; fp16 subnormals there cost < 2^-38 of the largest weight).
__device__ __forceinline__ void dev_pack_frag_s(int bid, const float* __restrict__ W, int F, int KS,
                              const PackHeader* __restrict__ hdr, uint4* __restrict__ wsh,
                              uint4* __restrict__ wsl) {
  int idx = bid * 256 + threadIdx.x;  // (s, ct, lane)
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

// Head-mean fragments (k_lone): B[k = f][n] = mean_h W[h C + n][f] * 2^kb,
// k-step s covers features 32 s .. 32 s + 31 (8 per lane group), lo unscaled.
__device__ __forceinline__ void dev_pack_wbar(int bid, const float* __restrict__ W, int F, int KB,
                            const PackHeader* __restrict__ hdr, uint4* __restrict__ wbh,
                            uint4* __restrict__ wbl) {
  int idx = bid * 256 + threadIdx.x;  // (s, ct, lane)
  if (idx >= KB * 4 * 64) return;
  int lane = idx & 63, ct = (idx >> 6) & 3, s = idx >> 8;
  int n = ct * 16 + (lane & 15);
  const float sc = hdr->wb_scale;
  union { uint4 v; _Float16 h[8]; } hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int f = 32 * s + 8 * (lane >> 4) + j;
    float v = 0.f;
    if (f < F) {
      float acc = 0.f;
#pragma unroll
      for (int h = 0; h < H; ++h) acc += W[size_t(h * C + n) * F + f];
      v = acc * (1.0f / H) * sc;
    }
    _Float16 hv = (_Float16)v;
    hi.h[j] = hv;
    lo.h[j] = (_Float16)(v - (float)hv);
  }
  wbh[idx] = hi.v;
  wbl[idx] = lo.v;
}

// Head-mean fragments in the logits pass's lane order (k_logits_lone): lane
// group g of k-step t holds, at positions j = 0..7, feature 32 t + 4 g + j
// (j < 4) or 32 t + 16 + 4 g + j - 4 (j >= 4) -- exactly the features that
// lane group's fp32 logits loads of k-steps 2 t and 2 t + 1 hold.
__device__ __forceinline__ void dev_pack_wbar_perm(int bid, const float* __restrict__ W, int F, int KB,
                                 const PackHeader* __restrict__ hdr, uint4* __restrict__ wph,
                                 uint4* __restrict__ wpl) {
  int idx = bid * 256 + threadIdx.x;  // (t, ct, lane)
  if (idx >= KB * 4 * 64) return;
  int lane = idx & 63, ct = (idx >> 6) & 3, t = idx >> 8;
  int n = ct * 16 + (lane & 15), g = lane >> 4;
  const float sc = hdr->wb_scale;
  union { uint4 v; _Float16 h[8]; } hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int f = 32 * t + 4 * g + j + (j >= 4 ? 12 : 0);
    float v = 0.f;
    if (f < F) {
      float acc = 0.f;
#pragma unroll
      for (int h = 0; h < H; ++h) acc += W[size_t(h * C + n) * F + f];
      v = acc * (1.0f / H) * sc;
    }
    _Float16 hv = (_Float16)v;
    hi.h[j] = hv;
    lo.h[j] = (_Float16)(v - (float)hv);
  }
  wph[idx] = hi.v;
  wpl[idx] = lo.v;
}

// [U | V] fragments (one 16-column tile: column n = q of uv, K = features),
// power-of-two scaled by max |uv| -> [2^13, 2^14), f16 hi / lo, in the lane
// order of k_pack_wbar_perm (fp32 logits pass) and in the plain order of
// k_pack_wbar (bf16 logits pass).  One block: the max, then the fragments.
__device__ __forceinline__ void dev_pack_uv_perm(const float* __restrict__ uv, int F, int Fu,
                                                      int KB, PackHeader* __restrict__ hdr,
                                                      uint4* __restrict__ uph,
                                                      uint4* __restrict__ upl,
                                                      uint4* __restrict__ ush,
                                                      uint4* __restrict__ usl) {
  __shared__ float red[256];
  const int t = threadIdx.x;
  float m = 0.f;
  for (int i = t; i < 2 * H * Fu; i += 256) m = fmaxf(m, fabsf(uv[i]));
  red[t] = m;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (t < s) red[t] = fmaxf(red[t], red[t + s]);
    __syncthreads();
  }
  const int ku = scale_exp(red[0]);
  const float sc = ldexpf(1.0f, ku);
  if (t == 0) {
    hdr->uv_scale = sc;
    hdr->uv_unscale = ldexpf(1.0f, -ku);
  }
  for (int idx = t; idx < 2 * KB * 64; idx += 256) {  // (order, k-step, lane)
    const bool plain = idx >= KB * 64;
    const int i = plain ? idx - KB * 64 : idx;
    const int lane = i & 63, kt = i >> 6;
    const int n = lane & 15, g = lane >> 4;
    union { uint4 v; _Float16 h[8]; } hi, lo;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int f = plain ? 32 * kt + 8 * g + j : 32 * kt + 4 * g + j + (j >= 4 ? 12 : 0);
      const float v = f < F ? uv[n * Fu + f] * sc : 0.f;
      const _Float16 hv = (_Float16)v;
      hi.h[j] = hv;
      lo.h[j] = (_Float16)(v - (float)hv);
    }
    (plain ? ush : uph)[i] = hi.v;
    (plain ? usl : upl)[i] = lo.v;
  }
}

// The pack in two launches (the seven kernels above as block ranges; round 5:
// seven small launches cost ~50 us per layer and step):
//   stage 1 (1024-thread blocks): block 0 the W scales, blocks 1.. U / V
//   stage 2 (256-thread blocks): fragments (need the scales) and [U | V]
//           fragments (need U / V), by block range
struct PackArgs {
  const float* W; const float* as; const float* ad; int F, Fp, Fu, KS, KB;
  PackHeader* hdr; float* uv;
  uint4 *whi, *wlo, *wsh, *wsl, *wbh, *wbl, *wph, *wpl, *uph, *upl, *ush, *usl;
};

__global__ void __launch_bounds__(1024) k_pack_stage1(PackArgs a) {
  if (blockIdx.x == 0) dev_wmax(a.W, a.F, a.hdr);
  else dev_pack_uv(a.W, a.as, a.ad, a.F, a.Fu, a.uv, int(blockIdx.x) - 1);
}

__global__ void __launch_bounds__(256) k_pack_stage2(PackArgs a) {
  const int nfr = (a.KS * 4 * 64 + 255) / 256, nwb = (a.KB * 4 * 64 + 255) / 256;
  int b = blockIdx.x;  // block-uniform ranges
  if (b < nfr) { dev_pack_frag(b, a.W, a.F, a.Fp, a.KS, a.hdr, a.whi, a.wlo); return; }
  b -= nfr;
  if (b < nfr) { dev_pack_frag_s(b, a.W, a.F, a.KS, a.hdr, a.wsh, a.wsl); return; }
  b -= nfr;
  if (b < nwb) { dev_pack_wbar(b, a.W, a.F, a.KB, a.hdr, a.wbh, a.wbl); return; }
  b -= nwb;
  if (b < nwb) { dev_pack_wbar_perm(b, a.W, a.F, a.KB, a.hdr, a.wph, a.wpl); return; }
  dev_pack_uv_perm(a.uv, a.F, a.Fu, a.KB, a.hdr, a.uph, a.upl, a.ush, a.usl);
}

// ---------------------------------------------------------------------------
// st[r][q] = sum_f x[r][f] * uv[q][f] (q < 2H) on v_mfma_f32_16x16x4_f32 with the
// 2H logit vectors stationary in registers (KSM k-steps of 16 features) and
// all KSM x loads of a 16-row tile issued before the first MFMA.  Lane group
// g = l >> 4 reads features 16 s + 4 g .. +3 of row l & 15; MFMA u of k-step
// s pairs them with uv[l & 15][16 s + 4 g + u]: the k order inside a k-step
// is permuted identically on both operands, so the sums are exact fp32 FMA
// chains.  Rows must be 4-element aligned (host-checked).
template <int KSM, typename XT>
__global__ void __launch_bounds__(256) k_logits_s(const typename XT::T* __restrict__ x,
                                                  int64_t rows, int F, int64_t ldx,
                                                  const float* __restrict__ uv, int Fu,
                                                  float* __restrict__ st,
                                                  float* __restrict__ xmax) {
  const int lane = threadIdx.x & 63;
  const int rl = lane & 15, g = lane >> 4;
  float am = 0.f;  // max |x| over the values this lane loaded (xmax != NULL)
  const int64_t wave = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nwave = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t tiles = (rows + 15) / 16;
  const int ksf = F / 16;         // k-steps fully inside the row
  const int kst = (F + 15) / 16;  // including the ragged tail
  f32x4 b[KSM];
#pragma unroll
  for (int s = 0; s < KSM; ++s)
    b[s] = s < kst ? *reinterpret_cast<const f32x4*>(uv + rl * Fu + 16 * s + 4 * g)
                   : f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t t = wave; t < tiles; t += nwave) {
    const int64_t row = t * 16 + rl;
    const typename XT::T* xr = x + (row < rows ? row : rows - 1) * ldx + 4 * g;
    f32x4 a[KSM];
#pragma unroll
    for (int s = 0; s < KSM; ++s) {
      if (s < ksf) {
        a[s] = load4<XT>(xr + 16 * s);
      } else if (s < kst) {  // ragged tail: guarded scalar loads (never past the row)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int f = 16 * s + 4 * g + u;
          a[s][u] = f < F ? xcvt(xr[16 * s + u]) : 0.f;
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
    if (lane == 0) atomic_max_nonneg(xmax, am);
  }
}

// Unaligned rows (any pitch / base): same product with scalar loads.
template <typename XT>
__global__ void __launch_bounds__(256) k_logits_u(const typename XT::T* __restrict__ x,
                                                  int64_t rows, int F, int64_t ldx,
                                                  const float* __restrict__ uv, int Fu,
                                                  float* __restrict__ st,
                                                  float* __restrict__ xmax) {
  const int lane = threadIdx.x & 63;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t wave = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nwave = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const int64_t tiles = (rows + 15) / 16;
  float am = 0.f;
  for (int64_t t = wave; t < tiles; t += nwave) {
    const int64_t row = t * 16 + rl;
    const typename XT::T* xr = x + (row < rows ? row : rows - 1) * ldx;
    f32x4 acc = {0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < F; k0 += 4) {
      const int f = k0 + g;
      const float xv = f < F ? xcvt(xr[f]) : 0.f;
      am = fmaxf(am, fabsf(xv));
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(xv, uv[rl * Fu + f], acc, 0, 0, 0);
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
    if (lane == 0) atomic_max_nonneg(xmax, am);
  }
}

template <typename XT>
gfd_status launch_logits_t(const typename XT::T* x, int64_t rows, int F, int64_t ldx,
                           const float* uv, int Fu, float* st, float* xmax, hipStream_t stream) {
  const int64_t tiles = (rows + 15) / 16;
  int64_t nb = (tiles + 3) / 4;
  const int64_t cap = int64_t(cu_count()) * 8;  // resident blocks; grid-stride beyond
  if (nb > cap) nb = cap;
  const uintptr_t a = reinterpret_cast<uintptr_t>(x);
  if (a % (4 * XT::kBytes) == 0 && ldx % 4 == 0) {
    if (F <= 176)
      k_logits_s<11, XT><<<int(nb), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st, xmax);
    else
      k_logits_s<16, XT><<<int(nb), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st, xmax);
  } else {
    k_logits_u<XT><<<int(nb), 256, 0, stream>>>(x, rows, F, ldx, uv, Fu, st, xmax);
  }
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

bool check_hc(int heads, int channels, int F) {
  return heads == H && channels == C && F >= 1 && F <= 256;
}

}  // namespace

namespace gfd {
namespace fwd {

gfd_status launch_logits(const void* x, int xdt, int64_t rows, int F, int64_t ldx,
                         const float* uv, int Fu, float* st, float* xmax, hipStream_t stream) {
  if (rows <= 0) return GFD_OK;
  if (xdt == GFD_DTYPE_BF16)
    return launch_logits_t<XBF16>(static_cast<const uint16_t*>(x), rows, F, ldx, uv, Fu, st,
                                  xmax, stream);
  return launch_logits_t<XF32>(static_cast<const float*>(x), rows, F, ldx, uv, Fu, st, xmax,
                               stream);
}

}  // namespace fwd
}  // namespace gfd

extern "C" {

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
  PackArgs a{weight, att_src, att_dst, F, L.Fp, L.Fu, L.KS, L.KB, hdr,
              reinterpret_cast<float*>(p + L.uv_off),
              reinterpret_cast<uint4*>(p + L.whi_off), reinterpret_cast<uint4*>(p + L.wlo_off),
              reinterpret_cast<uint4*>(p + L.wsh_off), reinterpret_cast<uint4*>(p + L.wsl_off),
              reinterpret_cast<uint4*>(p + L.wbh_off), reinterpret_cast<uint4*>(p + L.wbl_off),
              reinterpret_cast<uint4*>(p + L.wph_off), reinterpret_cast<uint4*>(p + L.wpl_off),
              reinterpret_cast<uint4*>(p + L.uph_off), reinterpret_cast<uint4*>(p + L.upl_off),
              reinterpret_cast<uint4*>(p + L.ush_off), reinterpret_cast<uint4*>(p + L.usl_off)};
  const int n_uv = 2 * H * L.Fu;
  k_pack_stage1<<<1 + (n_uv + 1023) / 1024, 1024, 0, stream>>>(a);
  GFD_LAUNCH_CHECK();
  const int nfr = (L.KS * 4 * 64 + 255) / 256, nwb = (L.KB * 4 * 64 + 255) / 256;
  k_pack_stage2<<<2 * nfr + 2 * nwb + 1, 256, 0, stream>>>(a);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

gfd_status gfd_gat_logits_ex(const void* x, int x_dtype, int64_t rows, int F, int64_t ldx,
                             const void* packed, int heads, int channels, float* st, float* xmax,
                             gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  if (x_dtype != GFD_DTYPE_F32 && x_dtype != GFD_DTYPE_BF16) return GFD_ERR_ARGUMENT;
  if (rows < 0 || (rows > 0 && (!x || !packed || !st)) || ldx < F) return GFD_ERR_ARGUMENT;
  PackLayout L = pack_layout(F);
  const float* uv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + L.uv_off);
  return launch_logits(x, x_dtype, rows, F, ldx, uv, L.Fu, st, xmax, stream);
}

gfd_status gfd_gat_logits(const void* x, int x_dtype, int64_t rows, int F, int64_t ldx,
                          const void* packed, int heads, int channels, float* st,
                          gfd_stream_t stream_) {
  return gfd_gat_logits_ex(x, x_dtype, rows, F, ldx, packed, heads, channels, st, nullptr,
                           stream_);
}

}  // extern "C"
