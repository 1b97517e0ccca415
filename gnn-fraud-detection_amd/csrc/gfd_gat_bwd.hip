// gfd_gat_bwd.hip -- GATConv backward for gfx950 (the autograd of PyG's
// GATConv dataflow that the reference runs at loss.backward(), train.py:142;
// formulas: SURVEY.md Appendix A).
//
//   k_gemm (fp32 MFMA 16x16x4, exact fp32 chains)  h = x W^T          [N, H*C]
//   k_bwd_dst   one wave per destination i (CSR): recompute alpha from the
//               saved (s, t, max, sum); dA = <g_i, h_jh>/H; softmax backward
//               -> dpre per message; dt_i; grad_bias
//   k_bwd_src   one wave per source j (CSC): ds_j = sum dpre; y_jh = sum
//               alpha_d g_i; dh_j = y/H + ds a_src + dt a_dst; grad_att_*
//   k_gemm      grad_x = dh W ;  grad_W = dh^T x (split-K over nodes)
#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int H = kHeads;
constexpr int C = kChannels;
constexpr int HC = H * C;

// ---------------------------------------------------------------------------
// Generic strided fp32 GEMM on v_mfma_f32_16x16x4_f32:
//   Cm(m, n) (+)= sum_k A(m, k) B(k, n);  X(r, c) = X[r * s_r + c * s_c]
// 64x64 block tile, BK = 16, 4 waves of 32x32; split-K over gridDim.z with
// float atomics into a zeroed C when gridDim.z > 1.
constexpr int GB = 64, GK = 16;

__global__ void __launch_bounds__(256) k_gemm(const float* __restrict__ A, int64_t sam,
                                              int64_t sak, const float* __restrict__ B,
                                              int64_t sbk, int64_t sbn, float* __restrict__ Cm,
                                              int64_t scm, int64_t scn, int64_t M, int64_t N,
                                              int64_t K, int64_t k_per_split) {
  __shared__ float As[GK][GB + 4];
  __shared__ float Bs[GK][GB + 4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t m0 = int64_t(blockIdx.x) * GB, n0 = int64_t(blockIdx.y) * GB;
  const int64_t kb = int64_t(blockIdx.z) * k_per_split;
  const int64_t ke = min(K, kb + k_per_split);
  const int wm = wave >> 1, wn = wave & 1;
  f32x4 acc[2][2];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u) acc[t][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t k0 = kb; k0 < ke; k0 += GK) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int idx = tid + 256 * q;  // 0..1023 = GK x GB
      // A tile: element (m = idx % GB, k = idx / GB)  [contiguous m when sam==1]
      // choose the mapping that keeps the unit-stride index in the lane
      int mm, kk;
      if (sak == 1) { kk = idx % GK; mm = idx / GK; } else { mm = idx % GB; kk = idx / GB; }
      const int64_t gm = m0 + mm, gk = k0 + kk;
      As[kk][mm] = (gm < M && gk < ke) ? A[gm * sam + gk * sak] : 0.f;
      int nn, kq;
      if (sbk == 1) { kq = idx % GK; nn = idx / GK; } else { nn = idx % GB; kq = idx / GB; }
      const int64_t gn = n0 + nn, gk2 = k0 + kq;
      Bs[kq][nn] = (gn < N && gk2 < ke) ? B[gk2 * sbk + gn * sbn] : 0.f;
    }
    __syncthreads();
#pragma unroll
    for (int kk = 0; kk < GK; kk += 4) {
      float a[2], b[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) a[t] = As[kk + (lane >> 4)][wm * 32 + t * 16 + (lane & 15)];
#pragma unroll
      for (int u = 0; u < 2; ++u) b[u] = Bs[kk + (lane >> 4)][wn * 32 + u * 16 + (lane & 15)];
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int u = 0; u < 2; ++u)
          acc[t][u] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[t], b[u], acc[t][u], 0, 0, 0);
    }
    __syncthreads();
  }
  const bool atomic = gridDim.z > 1;
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int u = 0; u < 2; ++u)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t gm = m0 + wm * 32 + t * 16 + (lane >> 4) * 4 + r;
        const int64_t gn = n0 + wn * 32 + u * 16 + (lane & 15);
        if (gm < M && gn < N) {
          float* p = Cm + gm * scm + gn * scn;
          if (atomic) atomicAdd(p, acc[t][u][r]);
          else *p = acc[t][u][r];
        }
      }
}

gfd_status gemm(const float* A, int64_t sam, int64_t sak, const float* B, int64_t sbk, int64_t sbn,
                float* Cm, int64_t scm, int64_t scn, int64_t M, int64_t N, int64_t K, int splits,
                hipStream_t stream) {
  if (M <= 0 || N <= 0) return GFD_OK;
  int64_t kps = (K + splits - 1) / splits;
  kps = (kps + GK - 1) / GK * GK;
  if (kps <= 0) kps = GK;
  int64_t z = (K + kps - 1) / kps;
  if (z < 1) z = 1;
  dim3 grid(unsigned((M + GB - 1) / GB), unsigned((N + GB - 1) / GB), unsigned(z));
  k_gemm<<<grid, 256, 0, stream>>>(A, sam, sak, B, sbk, sbn, Cm, scm, scn, M, N, K, kps);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

// ---------------------------------------------------------------------------
// dst-centric backward.  Lane layout for logits: lane = 8k + h.
__global__ void __launch_bounds__(256) k_bwd_dst(
    const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col, int64_t N,
    const float* __restrict__ st, const float* __restrict__ stats, const float* __restrict__ hproj,
    const float* __restrict__ g, float slope, float dp, uint64_t seed, float* __restrict__ dpre,
    float* __restrict__ alpha_d, float* __restrict__ dt, float* __restrict__ grad_bias) {
  const int lane = threadIdx.x & 63;
  const int h = lane & 7, kk = lane >> 3;
  const int64_t w0 = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nw = (int64_t(gridDim.x) * blockDim.x) >> 6;
  const float keep_scale = dp > 0.f ? 1.0f / (1.0f - dp) : 1.0f;
  float gb = 0.f;
  for (int64_t i = w0; i < N; i += nw) {
    const int e0 = rowptr[i], e1 = rowptr[i + 1];
    const float gc = g[i * C + lane];  // lane = channel
    gb += gc;
    const float t_h = st[i * 16 + H + h];
    const float m_h = stats[i * 16 + h];
    const float inv_h = 1.0f / (stats[i * 16 + H + h] + kSoftmaxEps);
    // pass 1: alpha, dA (grad wrt pre-dropout alpha), sum alpha*dA
    float adot = 0.f;
    for (int b = e0; b < e1; b += 8) {
      const int e = b + kk;
      float al = 0.f, keepf = 0.f;
      int j = 0;
      if (e < e1) {
        j = col[e];
        al = __expf(leaky(st[int64_t(j) * 16 + h] + t_h, slope) - m_h) * inv_h;
        keepf = (dp > 0.f) ? (dropout_keep(seed, uint32_t(e), uint32_t(h), dp) ? keep_scale : 0.f)
                           : 1.0f;
      }
      float my_da = 0.f;
      const int nk = min(8, e1 - b);
      for (int k = 0; k < nk; ++k) {
        const int jk = __builtin_amdgcn_readlane(j, 8 * k);
        const float* hr = hproj + int64_t(jk) * HC;
        float v[H];
#pragma unroll
        for (int hh = 0; hh < H; ++hh) v[hh] = gc * hr[hh * C + lane];
        // transposing reduce over 64 lanes: lane ends with head (lane >> 3)
#pragma unroll
        for (int step = 0; step < 3; ++step) {
          const int half = 4 >> step;
          const int mask = 32 >> step;
          const bool up = (lane & mask) != 0;
#pragma unroll
          for (int q = 0; q < half; ++q) {
            float send = up ? v[q] : v[q + half];
            float keep = up ? v[q + half] : v[q];
            v[q] = keep + __shfl_xor(send, mask);
          }
        }
        float r = v[0];
        r += __shfl_xor(r, 4);
        r += __shfl_xor(r, 2);
        r += __shfl_xor(r, 1);
        // lane 8k+h needs head h of edge k: lives in lanes 8h..8h+7
        const float got = __shfl(r, 8 * h);
        if (kk == k) my_da = got;
      }
      if (e < e1) {
        const float da = my_da * (1.0f / H) * keepf;  // d alpha (pre-dropout)
        adot = fmaf(al, da, adot);
        dpre[int64_t(e) * 8 + h] = da;                // stash, finished in pass 2
        alpha_d[int64_t(e) * 8 + h] = al * keepf;
      }
    }
    adot += __shfl_xor(adot, 8);
    adot += __shfl_xor(adot, 16);
    adot += __shfl_xor(adot, 32);
    // pass 2: de = alpha (dA - sum); dpre = de * leaky'(pre); dt_i = sum dpre
    float dts = 0.f;
    for (int b = e0; b < e1; b += 8) {
      const int e = b + kk;
      if (e < e1) {
        const int j = col[e];
        const float pre = st[int64_t(j) * 16 + h] + t_h;
        const float al = __expf(leaky(pre, slope) - m_h) * inv_h;
        const float da = dpre[int64_t(e) * 8 + h];
        const float d = al * (da - adot) * (pre > 0.f ? 1.0f : slope);
        dpre[int64_t(e) * 8 + h] = d;
        dts += d;
      }
    }
    dts += __shfl_xor(dts, 8);
    dts += __shfl_xor(dts, 16);
    dts += __shfl_xor(dts, 32);
    if (lane < 8) dt[i * 8 + lane] = dts;
  }
  if (grad_bias) atomicAdd(&grad_bias[lane], gb);
}

// src-centric: one wave per source node j; lane = channel c.
__global__ void __launch_bounds__(256) k_bwd_src(
    const int32_t* __restrict__ colptr, const int32_t* __restrict__ csc_dst,
    const int32_t* __restrict__ csc_eid, int64_t N, const float* __restrict__ dpre,
    const float* __restrict__ alpha_d, const float* __restrict__ dt, const float* __restrict__ g,
    const float* __restrict__ hproj, const float* __restrict__ att_src,
    const float* __restrict__ att_dst, float* __restrict__ dh, float* __restrict__ grad_as,
    float* __restrict__ grad_ad) {
  const int lane = threadIdx.x & 63;
  const int64_t w0 = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  const int64_t nw = (int64_t(gridDim.x) * blockDim.x) >> 6;
  float as[H], ad[H], gas[H], gad[H];
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    as[hh] = att_src[hh * C + lane];
    ad[hh] = att_dst[hh * C + lane];
    gas[hh] = 0.f;
    gad[hh] = 0.f;
  }
  for (int64_t j = w0; j < N; j += nw) {
    const int p0 = colptr[j], p1 = colptr[j + 1];
    float y[H], ds[H];
#pragma unroll
    for (int hh = 0; hh < H; ++hh) { y[hh] = 0.f; ds[hh] = 0.f; }
    for (int p = p0; p < p1; ++p) {
      const int e = csc_eid[p];
      const int i = csc_dst[p];
      const float gi = g[int64_t(i) * C + lane];
#pragma unroll
      for (int hh = 0; hh < H; ++hh) {
        y[hh] = fmaf(alpha_d[int64_t(e) * 8 + hh], gi, y[hh]);
        ds[hh] += dpre[int64_t(e) * 8 + hh];
      }
    }
    const float* hr = hproj + j * HC;
    float* dr = dh + j * HC;
#pragma unroll
    for (int hh = 0; hh < H; ++hh) {
      const float dtv = dt[j * 8 + hh];
      dr[hh * C + lane] = y[hh] * (1.0f / H) + ds[hh] * as[hh] + dtv * ad[hh];
      const float hv = hr[hh * C + lane];
      gas[hh] = fmaf(ds[hh], hv, gas[hh]);
      gad[hh] = fmaf(dtv, hv, gad[hh]);
    }
  }
#pragma unroll
  for (int hh = 0; hh < H; ++hh) {
    atomicAdd(&grad_as[hh * C + lane], gas[hh]);
    atomicAdd(&grad_ad[hh * C + lane], gad[hh]);
  }
}

int waves_grid(int64_t n) {
  int64_t blocks = (n + 3) / 4;
  if (blocks > 4096) blocks = 4096;
  if (blocks < 1) blocks = 1;
  return int(blocks);
}

}  // namespace

extern "C" {

size_t gfd_gat_bwd_workspace_size(int64_t N, int64_t M, int F, int heads, int channels) {
  if (heads != H || channels != C || F < 1 || F > 256 || N <= 0 || M < 0) return 0;
  Sizer s;
  s.take<float>(size_t(N) * HC);  // h
  s.take<float>(size_t(N) * HC);  // dh
  s.take<float>(size_t(M) * 8);   // dpre
  s.take<float>(size_t(M) * 8);   // alpha_d
  s.take<float>(size_t(N) * 8);   // dt
  return s.off;
}

gfd_status gfd_gat_bwd(const void* xv, int x_dtype, int64_t N, int F, int64_t ldx,
                       const int32_t* rowptr,
                       const int32_t* col, const int32_t* colptr, const int32_t* csc_dst,
                       const int32_t* csc_eid, int64_t M, const float* W, const float* att_src,
                       const float* att_dst, int heads, int channels, float slope, float dp,
                       uint64_t seed, const float* st, const float* stats, const float* g,
                       float* grad_x, float* grad_W, float* grad_as, float* grad_ad,
                       float* grad_bias, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (heads != H || channels != C || F < 1 || F > 256) return GFD_ERR_UNSUPPORTED;
  if (x_dtype != GFD_DTYPE_F32) return x_dtype == GFD_DTYPE_BF16 ? GFD_ERR_UNSUPPORTED : GFD_ERR_ARGUMENT;
  const float* x = static_cast<const float*>(xv);
  if (N <= 0 || M <= 0 || !x || !rowptr || !col || !colptr || !csc_dst || !csc_eid || !W ||
      !att_src || !att_dst || !st || !stats || !g || !grad_W || !grad_as || !grad_ad || ldx < F)
    return GFD_ERR_ARGUMENT;
  if (!(dp >= 0.f && dp < 1.f)) return GFD_ERR_ARGUMENT;
  if (ws_bytes < gfd_gat_bwd_workspace_size(N, M, F, heads, channels)) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  float* hproj = c.take<float>(size_t(N) * HC);
  float* dh = c.take<float>(size_t(N) * HC);
  float* dpre = c.take<float>(size_t(M) * 8);
  float* alpha_d = c.take<float>(size_t(M) * 8);
  float* dt = c.take<float>(size_t(N) * 8);
  if (!c.ok) return GFD_ERR_WORKSPACE;

  // h = x W^T  (A = x [N,F], B(k=f, n) = W[n][f])
  gfd_status s = gemm(x, ldx, 1, W, 1, F, hproj, HC, 1, N, HC, F, 1, stream);
  if (s != GFD_OK) return s;
  GFD_HIP_CHECK(hipMemsetAsync(grad_as, 0, sizeof(float) * HC, stream));
  GFD_HIP_CHECK(hipMemsetAsync(grad_ad, 0, sizeof(float) * HC, stream));
  if (grad_bias) GFD_HIP_CHECK(hipMemsetAsync(grad_bias, 0, sizeof(float) * C, stream));
  k_bwd_dst<<<waves_grid(N), 256, 0, stream>>>(rowptr, col, N, st, stats, hproj, g, slope, dp,
                                               seed, dpre, alpha_d, dt, grad_bias);
  GFD_LAUNCH_CHECK();
  k_bwd_src<<<waves_grid(N), 256, 0, stream>>>(colptr, csc_dst, csc_eid, N, dpre, alpha_d, dt, g,
                                               hproj, att_src, att_dst, dh, grad_as, grad_ad);
  GFD_LAUNCH_CHECK();
  // grad_W = dh^T x : M=HC (A(m,k=i) = dh[i][m]), N=F, K=N nodes, split-K
  GFD_HIP_CHECK(hipMemsetAsync(grad_W, 0, sizeof(float) * HC * F, stream));
  int splits = int(N / 4096);
  if (splits < 1) splits = 1;
  if (splits > 256) splits = 256;
  s = gemm(dh, 1, HC, x, ldx, 1, grad_W, F, 1, HC, F, N, splits, stream);
  if (s != GFD_OK) return s;
  if (grad_x) {
    // grad_x = dh W : A = dh [N, HC], B(k, n=f) = W[k][f]
    s = gemm(dh, HC, 1, W, F, 1, grad_x, F, 1, N, F, HC, 1, stream);
    if (s != GFD_OK) return s;
  }
  return GFD_OK;
}

}  // extern "C"
