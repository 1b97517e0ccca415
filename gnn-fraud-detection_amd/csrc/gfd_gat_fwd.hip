// gfd_gat_fwd.hip -- GATConv forward for gfx950 (PyG GATConv.forward, concat=False;
// called at /root/reference/src/models/gat.py:80 and tgn.py:94).
//
// Dataflow (aggregate-then-project; SURVEY.md §7 "hard parts"):
//   k_pack      W [H*C,F], att -> folded logit vectors U/V [2H][Fp] and the
//               bf16 hi/lo MFMA B-fragments of Wcat[(h,f)][c] = W[h*C+c][f] / H
//   k_logits    st[n] = (x_n.U_h, x_n.V_h)            -- one x read, 2H outputs
//   k_fused     per 16-destination tile:
//               phase A  per destination: two passes over its CSR segment --
//                        max of leaky(s_j + t_i), then p = exp(e - max),
//                        z_ih += p x_j (x rows gathered once, all 8 heads),
//                        z_ih /= sum p + 1e-16 -> Z tile in LDS (fp32)
//               phase B  out = Z . Wcat + bias on bf16 MFMA 16x16x32 with
//                        the 3-term split (Zhi.Whi + Zhi.Wlo + Zlo.Whi)
//   k_hub_*     destinations with > threshold messages are split into chunks
//               (partial max/sum/z per chunk) and merged before the tile.
#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int H = kHeads;
constexpr int C = kChannels;
constexpr int kTile = 16;          // destinations per fused block (MFMA M)
constexpr int kFusedThreads = 512; // 8 waves

struct PackLayout {
  int F, Fp, KP, KS;
  size_t uv_off, whi_off, wlo_off, bytes;
};

inline PackLayout pack_layout(int F) {
  PackLayout L;
  L.F = F;
  L.Fp = (F + 3) / 4 * 4;
  L.KP = H * L.Fp;          // multiple of 32
  L.KS = L.KP / 32;         // MFMA k-steps
  size_t o = 0;
  L.uv_off = o; o = align_up(o + sizeof(float) * 2 * H * L.Fp, 256);
  L.whi_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.wlo_off = o; o = align_up(o + sizeof(uint4) * size_t(L.KS) * 4 * 64, 256);
  L.bytes = o;
  return L;
}

// ---------------------------------------------------------------------------
__global__ void k_pack_uv(const float* __restrict__ W, const float* __restrict__ as,
                          const float* __restrict__ ad, int F, int Fp, float* __restrict__ uv) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;
  if (idx >= 2 * H * Fp) return;
  int q = idx / Fp, f = idx % Fp;
  int h = q % H;
  const float* a = (q < H ? as : ad) + h * C;
  float acc = 0.f;
  if (f < F) {
    for (int c = 0; c < C; ++c) acc = fmaf(a[c], W[size_t(h * C + c) * F + f], acc);
  }
  uv[idx] = acc;
}

__global__ void k_pack_frag(const float* __restrict__ W, int F, int Fp, int KS,
                            uint4* __restrict__ whi, uint4* __restrict__ wlo) {
  int idx = blockIdx.x * blockDim.x + threadIdx.x;  // (s, ct, lane)
  if (idx >= KS * 4 * 64) return;
  int lane = idx & 63, ct = (idx >> 6) & 3, s = idx >> 8;
  int n = ct * 16 + (lane & 15);
  union { uint4 v; uint16_t u[8]; } hi, lo;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    int k = 32 * s + 8 * (lane >> 4) + j;
    int h = k / Fp, f = k % Fp;
    float v = (f < F) ? W[size_t(h * C + n) * F + f] * (1.0f / H) : 0.f;
    uint16_t hb = bf16_bits(v);
    hi.u[j] = hb;
    lo.u[j] = bf16_bits(v - bf16_to_f32(hb));
  }
  whi[idx] = hi.v;
  wlo[idx] = lo.v;
}

// ---------------------------------------------------------------------------
// st[r][q] = sum_f x[r][f] * uv[q][f], q < 2H.  One wave per row; the 16 dot
// products are reduced with a transposing butterfly (17 shuffles per row).
template <int KF>
__global__ void __launch_bounds__(256) k_logits(const float* __restrict__ x, int64_t rows, int F,
                                                int64_t ldx, const float* __restrict__ uv, int Fp,
                                                float* __restrict__ st) {
  extern __shared__ __attribute__((aligned(16))) float s_uv[];  // [16][Fp]
  for (int i = threadIdx.x; i < 2 * H * Fp; i += blockDim.x) s_uv[i] = uv[i];
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nwave = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t r = wave; r < rows; r += nwave) {
    const float* xr = x + r * ldx;
    float xv[KF];
#pragma unroll
    for (int k = 0; k < KF; ++k) {
      int f = lane + 64 * k;
      xv[k] = f < F ? xr[f] : 0.f;
    }
    float v[16];
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < KF; ++k) {
        int f = lane + 64 * k;
        a = fmaf(xv[k], f < Fp ? s_uv[q * Fp + f] : 0.f, a);
      }
      v[q] = a;
    }
    // transposing butterfly: after xor 32,16,8,4 lane holds index q = lane>>2
#pragma unroll
    for (int step = 0; step < 4; ++step) {
      const int half = 8 >> step;        // 8,4,2,1 values kept
      const int mask = 32 >> step;       // 32,16,8,4
      const bool up = (lane & mask) != 0;
#pragma unroll
      for (int i = 0; i < half; ++i) {
        float send = up ? v[i] : v[i + half];
        float keep = up ? v[i + half] : v[i];
        v[i] = keep + __shfl_xor(send, mask);
      }
    }
    float t = v[0];
    t += __shfl_xor(t, 2);
    t += __shfl_xor(t, 1);
    if ((lane & 3) == 0) st[r * 16 + (lane >> 2)] = t;
  }
}

// ---------------------------------------------------------------------------
// Online part shared by the fused tile and the hub chunks.  Lane layout for
// the logits: lane = 8*k + h (edge k of a batch of 8, head h).
struct SegState {
  float m;     // max of head (lane & 7), valid in every lane after pass 1
  float ssum;  // denominator of head (lane & 7), reduced in every lane
};

template <int KF>
__device__ __forceinline__ SegState aggregate_segment(
    const float* __restrict__ x, int64_t ldx, int F, const int32_t* __restrict__ col, int e0,
    int e1, const float* __restrict__ st, float t_h, float slope, float dp, uint64_t seed,
    float (&acc)[H][KF]) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  // pass 1: max over the segment
  float m = -INFINITY;
  for (int b = e0; b < e1; b += 8) {
    int e = b + kk;
    if (e < e1) {
      int j = col[e];
      m = fmaxf(m, leaky(st[int64_t(j) * 16 + h] + t_h, slope));
    }
  }
  m = fmaxf(m, __shfl_xor(m, 8));
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  // pass 2: p = exp(e - max), z += p * x_j
#pragma unroll
  for (int hh = 0; hh < H; ++hh)
#pragma unroll
    for (int k = 0; k < KF; ++k) acc[hh][k] = 0.f;
  float ssum = 0.f;
  const float keep_scale = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
  for (int b = e0; b < e1; b += 8) {
    int e = b + kk;
    int j = 0;
    float p = 0.f;
    if (e < e1) {
      j = col[e];
      p = __expf(leaky(st[int64_t(j) * 16 + h] + t_h, slope) - m);
      ssum += p;
      if (dp > 0.f) p = dropout_keep(seed, uint32_t(e), uint32_t(h), dp) ? p * keep_scale : 0.f;
    }
    const int nk = min(8, e1 - b);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if (k < nk) {
        const int jk = __builtin_amdgcn_readlane(j, 8 * k);
        float pk[H];
#pragma unroll
        for (int hh = 0; hh < H; ++hh)
          pk[hh] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(p), 8 * k + hh));
        const float* xr = x + int64_t(jk) * ldx;
#pragma unroll
        for (int q = 0; q < KF; ++q) {
          const int f = lane + 64 * q;
          const float xv = f < F ? xr[f] : 0.f;
#pragma unroll
          for (int hh = 0; hh < H; ++hh) acc[hh][q] = fmaf(pk[hh], xv, acc[hh][q]);
        }
      }
    }
  }
  ssum += __shfl_xor(ssum, 8);
  ssum += __shfl_xor(ssum, 16);
  ssum += __shfl_xor(ssum, 32);
  return {m, ssum};
}

// ---------------------------------------------------------------------------
template <int KF>
__global__ void __launch_bounds__(kFusedThreads) k_fused(
    const float* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ rowptr,
    const int32_t* __restrict__ col, int64_t num_dst, int64_t dst_offset,
    const float* __restrict__ st, const uint4* __restrict__ whi, const uint4* __restrict__ wlo,
    const float* __restrict__ bias, float slope, float dp, uint64_t seed,
    const int32_t* __restrict__ hub_rank, const float* __restrict__ zhub,
    float* __restrict__ out, float* __restrict__ stats) {
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int KP = H * Fp;
  const int ZS = KP + 4;                  // padded row stride (bank spread)
  float* Z = smem;                        // [kTile][ZS]
  float* red = smem + kTile * ZS;         // [4][64][4] partials of the upper K half
  const int lane = threadIdx.x & 63;
  const int wave = wave_uniform(threadIdx.x >> 6);
  const int64_t tile0 = int64_t(blockIdx.x) * kTile;

  // ---- phase A: aggregate two destinations per wave into the Z tile ----
  for (int rr = 0; rr < 2; ++rr) {
    const int r = wave * 2 + rr;
    const int64_t i = tile0 + r;
    float* zr = Z + r * ZS;
    if (i >= num_dst) {
      for (int k = lane; k < KP; k += 64) zr[k] = 0.f;
      continue;
    }
    const int hr = hub_rank ? hub_rank[i] : -1;
    if (hr >= 0) {  // merged by k_hub_merge
      const float* src = zhub + int64_t(hr) * KP;
      for (int k = lane; k < KP; k += 64) zr[k] = src[k];
      continue;
    }
    const int e0 = rowptr[i], e1 = rowptr[i + 1];
    const int64_t gi = dst_offset + i;
    const float t_h = st[gi * 16 + H + (lane & 7)];
    float acc[H][KF];
    SegState S = aggregate_segment<KF>(x, ldx, F, col, e0, e1, st, t_h, slope, dp, seed, acc);
    const float inv_lane = 1.0f / (S.ssum + kSoftmaxEps);
    if (stats && lane < 8) {
      stats[i * 16 + lane] = S.m;
      stats[i * 16 + 8 + lane] = S.ssum;
    }
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
      const float inv = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(inv_lane), hh));
#pragma unroll
      for (int q = 0; q < KF; ++q) {
        const int f = lane + 64 * q;
        if (f < Fp) zr[hh * Fp + f] = acc[hh][q] * inv;
      }
    }
  }
  __syncthreads();

  // ---- phase B: out[16 x 64] = Z[16 x KP] . Wcat[KP x 64] on MFMA ----
  const int ct = wave & 3, kh = wave >> 2;
  const int KS = KP / 32;
  const int s0 = kh ? KS / 2 : 0, s1 = kh ? KS : KS / 2;
  f32x4 accv = {0.f, 0.f, 0.f, 0.f};
  const int arow = lane & 15, akg = lane >> 4;
  for (int s = s0; s < s1; ++s) {
    const float* zp = Z + arow * ZS + 32 * s + 8 * akg;
    float a8[8];
    *reinterpret_cast<float4*>(a8) = *reinterpret_cast<const float4*>(zp);
    *reinterpret_cast<float4*>(a8 + 4) = *reinterpret_cast<const float4*>(zp + 4);
    bf16x8 ahi, alo;
    split8(a8, ahi, alo);
    const uint4 bh = whi[(s * 4 + ct) * 64 + lane];
    const uint4 bl = wlo[(s * 4 + ct) * 64 + lane];
    const bf16x8 bhi = *reinterpret_cast<const bf16x8*>(&bh);
    const bf16x8 blo = *reinterpret_cast<const bf16x8*>(&bl);
    accv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, bhi, accv, 0, 0, 0);
    accv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ahi, blo, accv, 0, 0, 0);
    accv = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo, bhi, accv, 0, 0, 0);
  }
  if (kh) *reinterpret_cast<f32x4*>(red + (ct * 64 + lane) * 4) = accv;
  __syncthreads();
  if (!kh) {
    accv += *reinterpret_cast<const f32x4*>(red + (ct * 64 + lane) * 4);
    const int n = ct * 16 + (lane & 15);
    const float b = bias ? bias[n] : 0.f;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int64_t i = tile0 + (lane >> 4) * 4 + q;
      if (i < num_dst) out[i * C + n] = accv[q] + b;
    }
  }
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
  const int64_t gi = dst_offset + ck.w;
  const float t_h = st[gi * 16 + H + (lane & 7)];
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

// Merge the chunks of each hub: M = max m_c, S = sum S_c e^(m_c - M),
// z = sum z_c e^(m_c - M) / (S + eps).  One wave per hub.
__global__ void __launch_bounds__(256) k_hub_merge(const float* __restrict__ part, int Fp,
                                                   const int32_t* __restrict__ chunk_ptr,
                                                   const int32_t* __restrict__ hub_dst,
                                                   int64_t num_hubs, float* __restrict__ zhub,
                                                   float* __restrict__ stats) {
  const int lane = threadIdx.x & 63;
  const int64_t hb = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  if (hb >= num_hubs) return;
  const int KP = H * Fp;
  const int c0 = chunk_ptr[hb], c1 = chunk_ptr[hb + 1];
  // lanes 0..7 own heads; everyone computes M and S for head (lane & 7)
  const int h = lane & 7;
  float M = -INFINITY;
  for (int c = c0; c < c1; ++c) M = fmaxf(M, part[int64_t(c) * (16 + KP) + h]);
  float S = 0.f;
  for (int c = c0; c < c1; ++c) {
    const float* pr = part + int64_t(c) * (16 + KP);
    S += pr[8 + h] * __expf(pr[h] - M);
  }
  if (stats && lane < 8) {
    const int64_t i = hub_dst[hb];
    stats[i * 16 + lane] = M;
    stats[i * 16 + 8 + lane] = S;
  }
  float* zr = zhub + hb * KP;
  for (int k = lane; k < KP; k += 64) {
    const int hh = k / Fp;
    const float Mh = __shfl(M, hh);
    const float inv = 1.0f / (__shfl(S, hh) + kSoftmaxEps);
    float z = 0.f;
    for (int c = c0; c < c1; ++c) {
      const float* pr = part + int64_t(c) * (16 + KP);
      z = fmaf(pr[16 + k], __expf(pr[hh] - Mh), z);
    }
    zr[k] = z * inv;
  }
}

inline int kf_for(int F) { return (F + 63) / 64; }

size_t fused_smem(int Fp) { return sizeof(float) * (kTile * (H * Fp + 4) + 4 * 64 * 4); }

template <int KF>
gfd_status launch_logits(const float* x, int64_t rows, int F, int64_t ldx, const float* uv, int Fp,
                         float* st, hipStream_t stream) {
  if (rows <= 0) return GFD_OK;
  int64_t blocks = (rows + 3) / 4;
  if (blocks > 8192) blocks = 8192;
  k_logits<KF><<<int(blocks), 256, sizeof(float) * 16 * Fp, stream>>>(x, rows, F, ldx, uv, Fp, st);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

template <int KF>
gfd_status launch_aggregate(const float* x, int F, int Fp, int64_t ldx, const int32_t* rowptr,
                            const int32_t* col, int64_t num_dst, int64_t dst_offset,
                            const float* st, const PackLayout& L, const char* packed,
                            const float* bias, float slope, float dp, uint64_t seed,
                            const int32_t* hub_rank, const int32_t* hub_chunk,
                            const int32_t* hub_chunk_ptr, const int32_t* hub_dst,
                            int64_t num_hubs, int64_t num_chunks, int stages, float* out,
                            float* stats, float* part, float* zhub, hipStream_t stream) {
  const int KP = H * Fp;
  if (num_hubs > 0 && (stages & GFD_STAGE_HUBS)) {
    int64_t blocks = (num_chunks + 3) / 4;
    k_hub_partial<KF><<<int(blocks), 256, 0, stream>>>(x, F, Fp, ldx, col, dst_offset, st, slope,
                                                       dp, seed,
                                                       reinterpret_cast<const int4*>(hub_chunk),
                                                       num_chunks, part);
    GFD_LAUNCH_CHECK();
    k_hub_merge<<<int((num_hubs + 3) / 4), 256, 0, stream>>>(part, Fp, hub_chunk_ptr, hub_dst,
                                                             num_hubs, zhub, stats);
    GFD_LAUNCH_CHECK();
  }
  (void)KP;
  if (!(stages & GFD_STAGE_TILES)) return GFD_OK;
  const int64_t tiles = (num_dst + kTile - 1) / kTile;
  if (tiles > 0x7fffffff) return GFD_ERR_UNSUPPORTED;
  const uint4* whi = reinterpret_cast<const uint4*>(packed + L.whi_off);
  const uint4* wlo = reinterpret_cast<const uint4*>(packed + L.wlo_off);
  k_fused<KF><<<int(tiles), kFusedThreads, fused_smem(Fp), stream>>>(
      x, F, Fp, ldx, rowptr, col, num_dst, dst_offset, st, whi, wlo, bias, slope, dp, seed,
      num_hubs > 0 ? hub_rank : nullptr, zhub, out, stats);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

bool check_hc(int heads, int channels, int F) {
  return heads == H && channels == C && F >= 1 && F <= 256;
}

}  // namespace

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
  int n_uv = 2 * H * L.Fp;
  k_pack_uv<<<(n_uv + 255) / 256, 256, 0, stream>>>(weight, att_src, att_dst, F, L.Fp,
                                                    reinterpret_cast<float*>(p + L.uv_off));
  GFD_LAUNCH_CHECK();
  int n_fr = L.KS * 4 * 64;
  k_pack_frag<<<(n_fr + 255) / 256, 256, 0, stream>>>(weight, F, L.Fp, L.KS,
                                                      reinterpret_cast<uint4*>(p + L.whi_off),
                                                      reinterpret_cast<uint4*>(p + L.wlo_off));
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

gfd_status gfd_gat_logits(const float* x, int64_t rows, int F, int64_t ldx, const void* packed,
                          int heads, int channels, float* st, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  if (rows < 0 || (rows > 0 && (!x || !packed || !st)) || ldx < F) return GFD_ERR_ARGUMENT;
  PackLayout L = pack_layout(F);
  const float* uv = reinterpret_cast<const float*>(static_cast<const char*>(packed) + L.uv_off);
  switch (kf_for(F)) {
    case 1: return launch_logits<1>(x, rows, F, ldx, uv, L.Fp, st, stream);
    case 2: return launch_logits<2>(x, rows, F, ldx, uv, L.Fp, st, stream);
    case 3: return launch_logits<3>(x, rows, F, ldx, uv, L.Fp, st, stream);
    default: return launch_logits<4>(x, rows, F, ldx, uv, L.Fp, st, stream);
  }
}

size_t gfd_gat_fwd_workspace_size(int64_t num_nodes, int64_t num_dst, int F, int heads,
                                  int channels, int64_t num_hubs, int64_t num_chunks) {
  if (!check_hc(heads, channels, F)) return 0;
  (void)num_dst;
  PackLayout L = pack_layout(F);
  Sizer s;
  s.take<char>(L.bytes);                              // packed weights (gfd_gat_fwd only)
  s.take<float>(size_t(num_nodes) * 16);              // st (gfd_gat_fwd when st == NULL)
  s.take<float>(size_t(num_chunks) * (16 + L.KP));    // hub partials
  s.take<float>(size_t(num_hubs) * L.KP);             // merged hub z rows
  return s.off;
}

static gfd_status aggregate_impl(const float* x, int64_t N, int F, int64_t ldx,
                                 const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                                 int64_t dst_offset, const float* st, const void* packed,
                                 const float* bias, float slope, float dp, uint64_t seed,
                                 const int32_t* hub_rank, const int32_t* hub_chunk,
                                 const int32_t* hub_chunk_ptr, const int32_t* hub_dst,
                                 int64_t num_hubs, int64_t num_chunks, int stages, float* out,
                                 float* stats, float* part, float* zhub, hipStream_t stream) {
  PackLayout L = pack_layout(F);
  const char* pk = static_cast<const char*>(packed);
  switch (kf_for(F)) {
#define GFD_AGG(KF)                                                                              \
  case KF:                                                                                       \
    return launch_aggregate<KF>(x, F, L.Fp, ldx, rowptr, col, num_dst, dst_offset, st, L, pk,    \
                                bias, slope, dp, seed, hub_rank, hub_chunk, hub_chunk_ptr,       \
                                hub_dst, num_hubs, num_chunks, stages, out, stats, part, zhub,   \
                                stream);
    GFD_AGG(1)
    GFD_AGG(2)
    GFD_AGG(3)
    GFD_AGG(4)
#undef GFD_AGG
    default: return GFD_ERR_UNSUPPORTED;
  }
  (void)N;
}

static gfd_status check_agg_args(const float* x, int64_t N, int F, int64_t ldx,
                                 const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                                 int64_t dst_offset, float dp, const int32_t* hub_rank,
                                 const int32_t* hub_chunk, const int32_t* hub_chunk_ptr,
                                 const int32_t* hub_dst, int64_t num_hubs, int64_t num_chunks,
                                 float* out) {
  if (N <= 0 || num_dst < 0 || dst_offset < 0 || dst_offset + num_dst > N) return GFD_ERR_ARGUMENT;
  if (!x || !rowptr || !col || !out || ldx < F) return GFD_ERR_ARGUMENT;
  if (!(dp >= 0.f && dp < 1.f)) return GFD_ERR_ARGUMENT;
  if (num_hubs < 0 || num_chunks < 0) return GFD_ERR_ARGUMENT;
  if (num_hubs > 0 && (!hub_rank || !hub_chunk || !hub_chunk_ptr || !hub_dst || num_chunks <= 0))
    return GFD_ERR_ARGUMENT;
  return GFD_OK;
}

gfd_status gfd_gat_aggregate(const float* x, int64_t N, int F, int64_t ldx, const int32_t* rowptr,
                             const int32_t* col, int64_t num_dst, int64_t dst_offset,
                             const float* st, const void* packed, const float* bias, int heads,
                             int channels, float slope, float dp, uint64_t seed,
                             const int32_t* hub_rank, const int32_t* hub_chunk,
                             const int32_t* hub_chunk_ptr, const int32_t* hub_dst,
                             int64_t num_hubs, int64_t num_chunks, int stages, float* out,
                             float* stats, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  gfd_status a = check_agg_args(x, N, F, ldx, rowptr, col, num_dst, dst_offset, dp, hub_rank,
                                hub_chunk, hub_chunk_ptr, hub_dst, num_hubs, num_chunks, out);
  if (a != GFD_OK) return a;
  if (!st || !packed || stages < 1 || stages > 3) return GFD_ERR_ARGUMENT;
  if (num_dst == 0) return GFD_OK;
  PackLayout L = pack_layout(F);
  Carve c(ws, ws_bytes);
  float* part = nullptr;
  float* zhub = nullptr;
  if (num_hubs > 0) {
    part = c.take<float>(size_t(num_chunks) * (16 + L.KP));
    zhub = c.take<float>(size_t(num_hubs) * L.KP);
    if (!c.ok) return GFD_ERR_WORKSPACE;
  }
  return aggregate_impl(x, N, F, ldx, rowptr, col, num_dst, dst_offset, st, packed, bias, slope,
                        dp, seed, hub_rank, hub_chunk, hub_chunk_ptr, hub_dst, num_hubs,
                        num_chunks, stages, out, stats, part, zhub, stream);
}

gfd_status gfd_gat_fwd(const float* x, int64_t N, int F, int64_t ldx, const int32_t* rowptr,
                       const int32_t* col, const float* weight, const float* att_src,
                       const float* att_dst, const float* bias, int heads, int channels,
                       float slope, float dp, uint64_t seed, const int32_t* hub_rank,
                       const int32_t* hub_chunk, const int32_t* hub_chunk_ptr,
                       const int32_t* hub_dst, int64_t num_hubs, int64_t num_chunks, float* out,
                       float* st, float* stats, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!check_hc(heads, channels, F)) return GFD_ERR_UNSUPPORTED;
  gfd_status a = check_agg_args(x, N, F, ldx, rowptr, col, N, 0, dp, hub_rank, hub_chunk,
                                hub_chunk_ptr, hub_dst, num_hubs, num_chunks, out);
  if (a != GFD_OK) return a;
  if (!weight || !att_src || !att_dst) return GFD_ERR_ARGUMENT;
  if (ws_bytes < gfd_gat_fwd_workspace_size(N, N, F, heads, channels, num_hubs, num_chunks))
    return GFD_ERR_WORKSPACE;
  PackLayout L = pack_layout(F);
  Carve c(ws, ws_bytes);
  void* packed = c.take<char>(L.bytes);
  float* st_ws = c.take<float>(size_t(N) * 16);
  float* part = c.take<float>(size_t(num_chunks) * (16 + L.KP));
  float* zhub = c.take<float>(size_t(num_hubs) * L.KP);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  if (st == nullptr) st = st_ws;
  gfd_status s = gfd_gat_pack_weights(weight, att_src, att_dst, F, heads, channels, packed, stream_);
  if (s != GFD_OK) return s;
  s = gfd_gat_logits(x, N, F, ldx, packed, heads, channels, st, stream_);
  if (s != GFD_OK) return s;
  return aggregate_impl(x, N, F, ldx, rowptr, col, N, 0, st, packed, bias, slope, dp, seed,
                        hub_rank, hub_chunk, hub_chunk_ptr, hub_dst, num_hubs, num_chunks,
                        GFD_STAGE_ALL, out, stats, part, zhub, stream);
}

}  // extern "C"
