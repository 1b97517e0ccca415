// gfd_epilogue.hip -- the training-mode layer body of the reference
// (/root/reference/src/models/gat.py:82-91, tgn.py:96-105):
//   z = BatchNorm1d(y) with batch statistics, r = relu(z), d = dropout(r, p),
//   h' = h + d (residual) or d,
// forward and backward in four kernels instead of ATen's chain of BN
// statistics / normalise / relu / dropout (mask + scale) / add launches and
// their [N, 64] intermediates.
//
//   k_col_stats   per-channel sum and sum of squares of y (forward) or of
//                 (dz, dz * xhat) (backward): deterministic two-level
//                 reduction (fixed block partials, then one block), no float
//                 atomics
//   k_bn_fwd      normalise, relu, dropout, residual; h' written once
//   k_bn_bwd      dy = gamma * invstd / N * (N dz - sum dz - xhat sum dz xhat),
//                 dz = dh' * mask / (1 - p) * [z > 0] recomputed from y
// The dropout mask is counter-based (splitmix64 of seed, row * C + channel):
// the backward regenerates it; it is not torch's RNG stream (the reference's
// F.dropout), the same distribution.
#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int kC = kChannels;  // 64 channels
constexpr int kEB = 256;       // threads per block: 4 rows x 64 channels per pass
constexpr int kParts = 1024;   // first-level partial blocks

// part[b][0..63] = sum of a, part[b][64..127] = sum of b over this block's rows
// mode 0: (y, y^2); mode 1/2: (g, g * xhat) with g = dz recomputed from y
// (mode 1 through the relu, mode 2 without) and xhat = (y - mean) * invstd
__global__ void __launch_bounds__(kEB) k_col_stats(
    const float* __restrict__ y, const float* __restrict__ gout, const float* __restrict__ mean,
    const float* __restrict__ invstd, const float* __restrict__ gamma,
    const float* __restrict__ beta, int64_t N, int mode, float p, uint64_t seed,
    double* __restrict__ part) {
  __shared__ double sa[kEB], sb[kEB];
  const int c = threadIdx.x & (kC - 1), r0 = threadIdx.x >> 6;
  const float keep = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  // four rows' loads in flight per thread (four accumulator pairs, combined in
  // a fixed order: the sums stay deterministic)
  double aa[4] = {0.0, 0.0, 0.0, 0.0}, bb[4] = {0.0, 0.0, 0.0, 0.0};
  const int64_t stride = int64_t(gridDim.x) * 4;
  auto row = [&](int64_t r, int u) {
    const float v = y[r * kC + c];
    if (mode == 0) {
      aa[u] += v;
      bb[u] += double(v) * v;
    } else {
      const float xh = (v - mean[c]) * invstd[c];
      const float z = xh * gamma[c] + beta[c];
      float g = gout[r * kC + c];
      if (p > 0.f) g = dropout_keep(seed, uint32_t(r * kC + c), 0, p) ? g * keep : 0.f;
      if (mode == 1) g = z > 0.f ? g : 0.f;
      aa[u] += g;
      bb[u] += double(g) * xh;
    }
  };
  int64_t r = blockIdx.x * 4 + r0;
  for (; r + 3 * stride < N; r += 4 * stride) {
#pragma unroll
    for (int u = 0; u < 4; ++u) row(r + u * stride, u);
  }
  for (; r < N; r += stride) row(r, 0);
  double a = (aa[0] + aa[1]) + (aa[2] + aa[3]);
  double b = (bb[0] + bb[1]) + (bb[2] + bb[3]);
  sa[threadIdx.x] = a;
  sb[threadIdx.x] = b;
  __syncthreads();
  if (threadIdx.x < kC) {
    for (int k = 1; k < 4; ++k) {
      a += sa[threadIdx.x + 64 * k];
      b += sb[threadIdx.x + 64 * k];
    }
    part[blockIdx.x * 2 * kC + c] = a;
    part[blockIdx.x * 2 * kC + kC + c] = b;
  }
}

// one block of 1024 threads: thread (g, c) sums partials g, g + 8, ... of
// column c (0..127: the a and b sums), then the 8 groups in order -- a fixed
// order whatever the partial count
__global__ void __launch_bounds__(1024) k_col_final(const double* __restrict__ part, int parts,
                                                    double* __restrict__ out) {
  __shared__ double red[8][2 * kC];
  const int c = threadIdx.x & (2 * kC - 1), g = threadIdx.x >> 7;
  double aa[4] = {0.0, 0.0, 0.0, 0.0};  // four loads in flight, fixed combination order
  int k = g;
  for (; k + 24 < parts; k += 32) {
#pragma unroll
    for (int u = 0; u < 4; ++u) aa[u] += part[(k + 8 * u) * 2 * kC + c];
  }
  for (; k < parts; k += 8) aa[0] += part[k * 2 * kC + c];
  red[g][c] = (aa[0] + aa[1]) + (aa[2] + aa[3]);
  __syncthreads();
  if (threadIdx.x < 2 * kC) {
    double t = 0.0;
    for (int k = 0; k < 8; ++k) t += red[k][c];
    out[c] = t;
  }
}

// batch mean / biased var -> mean, invstd; running stats (unbiased var) update
__global__ void __launch_bounds__(kC) k_bn_moments(const double* __restrict__ sums, int64_t N,
                                                   float eps, float momentum,
                                                   float* __restrict__ mean,
                                                   float* __restrict__ invstd,
                                                   float* __restrict__ run_mean,
                                                   float* __restrict__ run_var) {
  const int c = threadIdx.x;
  const double m = sums[c] / double(N);
  double v = sums[kC + c] / double(N) - m * m;
  if (v < 0.0) v = 0.0;
  mean[c] = float(m);
  invstd[c] = float(1.0 / sqrt(v + double(eps)));
  if (run_mean) run_mean[c] = (1.0f - momentum) * run_mean[c] + momentum * float(m);
  if (run_var)
    run_var[c] = (1.0f - momentum) * run_var[c] +
                 momentum * float(N > 1 ? v * double(N) / double(N - 1) : v);
}

__global__ void __launch_bounds__(kEB) k_bn_fwd(const float* __restrict__ y,
                                                const float* __restrict__ res, int64_t N,
                                                const float* __restrict__ mean,
                                                const float* __restrict__ invstd,
                                                const float* __restrict__ gamma,
                                                const float* __restrict__ beta, int relu, float p,
                                                uint64_t seed, float* __restrict__ out) {
  const int c = threadIdx.x & (kC - 1), r0 = threadIdx.x >> 6;
  const float keep = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  for (int64_t r = blockIdx.x * 4 + r0; r < N; r += int64_t(gridDim.x) * 4) {
    float z = (y[r * kC + c] - mean[c]) * invstd[c] * ga + be;
    if (relu) z = fmaxf(z, 0.f);
    if (p > 0.f) z = dropout_keep(seed, uint32_t(r * kC + c), 0, p) ? z * keep : 0.f;
    if (res) z += res[r * kC + c];
    out[r * kC + c] = z;
  }
}

__global__ void __launch_bounds__(kEB) k_bn_bwd(const float* __restrict__ y,
                                                const float* __restrict__ gout, int64_t N,
                                                const float* __restrict__ mean,
                                                const float* __restrict__ invstd,
                                                const float* __restrict__ gamma,
                                                const float* __restrict__ beta,
                                                const double* __restrict__ sums, int relu,
                                                float p, uint64_t seed, float* __restrict__ gy) {
  const int c = threadIdx.x & (kC - 1), r0 = threadIdx.x >> 6;
  const float keep = p > 0.f ? 1.0f / (1.0f - p) : 1.0f;
  const float ga = gamma ? gamma[c] : 1.f, be = beta ? beta[c] : 0.f;
  const float sg = float(sums[c] / double(N)), sgx = float(sums[kC + c] / double(N));
  const float k = ga * invstd[c];
  for (int64_t r = blockIdx.x * 4 + r0; r < N; r += int64_t(gridDim.x) * 4) {
    const float xh = (y[r * kC + c] - mean[c]) * invstd[c];
    const float z = xh * ga + be;
    float g = gout[r * kC + c];
    if (p > 0.f) g = dropout_keep(seed, uint32_t(r * kC + c), 0, p) ? g * keep : 0.f;
    if (relu) g = z > 0.f ? g : 0.f;
    gy[r * kC + c] = k * (g - sg - xh * sgx);
  }
}

__global__ void __launch_bounds__(kC) k_affine_grads(const double* __restrict__ s,
                                                     float* __restrict__ gg,
                                                     float* __restrict__ gb) {
  const int c = threadIdx.x;
  if (gb) gb[c] = float(s[c]);
  if (gg) gg[c] = float(s[kC + c]);
}

int egrid(int64_t N) {
  const int64_t g = (N + 3) / 4;
  return int(g < kParts ? (g < 1 ? 1 : g) : kParts);
}

}  // namespace

extern "C" {

size_t gfd_bn_workspace_size(void) { return sizeof(double) * (kParts * 2 * kC + 2 * kC) + 256; }

gfd_status gfd_bn_relu_fwd(const float* y, const float* residual, int64_t N, int channels,
                           const float* gamma, const float* beta, float eps, float momentum,
                           float* running_mean, float* running_var, int relu, float dropout_p,
                           uint64_t seed, float* out, float* mean, float* invstd, void* ws,
                           size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (channels != kC) return GFD_ERR_UNSUPPORTED;
  if (N <= 0 || !y || !out || !mean || !invstd || !(dropout_p >= 0.f && dropout_p < 1.f))
    return GFD_ERR_ARGUMENT;
  if (N * kC >= (int64_t(1) << 32)) return GFD_ERR_UNSUPPORTED;  // 32-bit mask counters
  Carve c(ws, ws_bytes);
  double* part = c.take<double>(kParts * 2 * kC);
  double* sums = c.take<double>(2 * kC);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  const int g = egrid(N);
  k_col_stats<<<g, kEB, 0, stream>>>(y, nullptr, nullptr, nullptr, nullptr, nullptr, N, 0, 0.f,
                                      0, part);
  GFD_LAUNCH_CHECK();
  k_col_final<<<1, 1024, 0, stream>>>(part, g, sums);
  GFD_LAUNCH_CHECK();
  k_bn_moments<<<1, kC, 0, stream>>>(sums, N, eps, momentum, mean, invstd, running_mean,
                                     running_var);
  GFD_LAUNCH_CHECK();
  k_bn_fwd<<<egrid(N) * 4, kEB, 0, stream>>>(y, residual, N, mean, invstd, gamma, beta, relu,
                                              dropout_p, seed, out);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

gfd_status gfd_bn_relu_bwd(const float* y, const float* grad_out, int64_t N, int channels,
                           const float* gamma, const float* beta, const float* mean,
                           const float* invstd, int relu, float dropout_p, uint64_t seed,
                           float* grad_y, float* grad_gamma, float* grad_beta, void* ws,
                           size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (channels != kC) return GFD_ERR_UNSUPPORTED;
  if (N <= 0 || !y || !grad_out || !mean || !invstd || !grad_y) return GFD_ERR_ARGUMENT;
  if (!gamma || !beta) return GFD_ERR_ARGUMENT;  // the affine BatchNorm of the reference
  Carve c(ws, ws_bytes);
  double* part = c.take<double>(kParts * 2 * kC);
  double* sums = c.take<double>(2 * kC);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  const int g = egrid(N);
  k_col_stats<<<g, kEB, 0, stream>>>(y, grad_out, mean, invstd, gamma, beta, N, relu ? 1 : 2,
                                      dropout_p, seed, part);
  GFD_LAUNCH_CHECK();
  k_col_final<<<1, 1024, 0, stream>>>(part, g, sums);
  GFD_LAUNCH_CHECK();
  k_bn_bwd<<<egrid(N) * 4, kEB, 0, stream>>>(y, grad_out, N, mean, invstd, gamma, beta, sums,
                                              relu, dropout_p, seed, grad_y);
  GFD_LAUNCH_CHECK();
  // grad_beta = sum dz, grad_gamma = sum dz * xhat (the same sums)
  if (grad_beta || grad_gamma) {
    k_affine_grads<<<1, kC, 0, stream>>>(sums, grad_gamma, grad_beta);
    GFD_LAUNCH_CHECK();
  }
  return GFD_OK;
}

}  // extern "C"
