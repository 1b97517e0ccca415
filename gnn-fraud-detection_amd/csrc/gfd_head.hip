// gfd_head.hip -- the TemporalGNN head of /root/reference/src/models/tgn.py:
// GRUCell(h, h0) (tgn.py:60, :108) followed by Linear(64 -> out) (tgn.py:63,
// :111), in one kernel per 16-row tile, so the [N, 192] gate pre-activations
// never reach HBM.
//
// PyTorch GRUCell semantics (gate blocks r, z, n of W_ih / W_hh [3C, C]):
//   r = sigmoid(x W_ir^T + b_ir + h W_hr^T + b_hr)
//   z = sigmoid(x W_iz^T + b_iz + h W_hz^T + b_hz)
//   n = tanh(x W_in^T + b_in + r * (h W_hn^T + b_hn))
//   h' = (1 - z) * n + z * h
// The reference always calls it with h0 = 0 (tgn.py:88-89), where the W_hh
// products vanish and only b_hh remains; h0 != NULL runs the second product.
//
// k_gru_head: one wave per 16-row tile (grid-stride), W_ih (and W_hh) in LDS
// in the B layout of v_mfma_f32_16x16x4_f32 (exact fp32 products and sums),
// 12 column tiles of 16 gate columns per product; lane (r, g) of the A operand
// loads features 16 s + 4 g .. +3 of row r (the k order inside each k-step is
// permuted identically on both operands).  Every gate of output column c sits
// in the same lane, so the update is register-local; the Linear head is a
// 16-lane DPP reduction per output.
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

constexpr int kHW = 8;     // waves per block
constexpr int kG = 3 * C;  // gate columns

__device__ __forceinline__ float sigmoidf(float v) { return 1.0f / (1.0f + __expf(-v)); }
// tanh(v) = 1 - 2 / (exp(2 v) + 1): saturates cleanly at +-1 for large |v|
__device__ __forceinline__ float tanh_fast(float v) { return 1.0f - 2.0f / (__expf(2.0f * v) + 1.0f); }

// sum over the 16 lanes of each DPP row (lanes 16 g .. 16 g + 15)
__device__ __forceinline__ float sum16(float v) {
  v += dpp_mov<0x121>(v);  // row_ror:1
  v += dpp_mov<0x122>(v);  // row_ror:2
  v += dpp_mov<0x124>(v);  // row_ror:4
  v += dpp_mov<0x128>(v);  // row_ror:8
  return v;
}

// acc += rows (16 x 64, lane layout above) . W^T for gate column tile ct
__device__ __forceinline__ void gate_mfma(const f32x4 (&a)[4], const f32x4* __restrict__ Ws,
                                          int ct, int lane, f32x4& acc) {
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const f32x4 b = Ws[(ct * 4 + s) * 64 + lane];
#pragma unroll
    for (int u = 0; u < 4; ++u)
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][u], b[u], acc, 0, 0, 0);
  }
}

__global__ void __launch_bounds__(kHW * 64) k_gru_head(
    const float* __restrict__ h, int64_t ldh, int64_t rows, const float* __restrict__ w_ih,
    const float* __restrict__ b_ih, const float* __restrict__ w_hh, const float* __restrict__ b_hh,
    const float* __restrict__ h0, int64_t ldh0, const float* __restrict__ w_out,
    const float* __restrict__ b_out, int n_out, float* __restrict__ h_new,
    float* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  // W*[(ct * 4 + s) * 64 + lane] = W[16 ct + (lane & 15)][16 s + 4 (lane >> 4) .. +3]
  f32x4* Wi = reinterpret_cast<f32x4*>(ssm);
  f32x4* Wh = Wi + 12 * 4 * 64;
  const int nw = h0 ? 2 : 1;
  for (int i = threadIdx.x; i < nw * 12 * 4 * 64; i += blockDim.x) {
    const int which = i / (12 * 4 * 64), j = i % (12 * 4 * 64);
    const int l = j & 63, s = (j >> 6) & 3, ct = j >> 8;
    const float* W = which ? w_hh : w_ih;
    Wi[i] = *reinterpret_cast<const f32x4*>(W + (16 * ct + (l & 15)) * C + 16 * s + 4 * (l >> 4));
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int rl = lane & 15, g = lane >> 4;
  const int64_t wave = int64_t(blockIdx.x) * kHW + (threadIdx.x >> 6);
  const int64_t nwave = int64_t(gridDim.x) * kHW;
  const int64_t tiles = (rows + 15) / 16;
  for (int64_t t = wave; t < tiles; t += nwave) {
    const int64_t row = t * 16 + rl;
    const int64_t rr = row < rows ? row : rows - 1;
    f32x4 a[4], a0[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      a[s] = *reinterpret_cast<const f32x4*>(h + rr * ldh + 16 * s + 4 * g);
      a0[s] = h0 ? *reinterpret_cast<const f32x4*>(h0 + rr * ldh0 + 16 * s + 4 * g)
                 : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    // output column c = 16 ct + rl of rows 4 g + q: every gate of c in this lane
    float hn[4][4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      f32x4 gr = {0.f, 0.f, 0.f, 0.f}, gz = gr, gn = gr, hr = gr, hz = gr, hh = gr;
      gate_mfma(a, Wi, ct, lane, gr);
      gate_mfma(a, Wi, 4 + ct, lane, gz);
      gate_mfma(a, Wi, 8 + ct, lane, gn);
      if (h0) {
        gate_mfma(a0, Wh, ct, lane, hr);
        gate_mfma(a0, Wh, 4 + ct, lane, hz);
        gate_mfma(a0, Wh, 8 + ct, lane, hh);
      }
      const int c = 16 * ct + rl;
      const float bir = b_ih ? b_ih[c] : 0.f, biz = b_ih ? b_ih[C + c] : 0.f,
                  bin = b_ih ? b_ih[2 * C + c] : 0.f;
      const float bhr = b_hh ? b_hh[c] : 0.f, bhz = b_hh ? b_hh[C + c] : 0.f,
                  bhn = b_hh ? b_hh[2 * C + c] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t orow = t * 16 + 4 * g + q;
        const float r = sigmoidf(gr[q] + bir + hr[q] + bhr);
        const float z = sigmoidf(gz[q] + biz + hz[q] + bhz);
        const float n = tanh_fast(gn[q] + bin + r * (hh[q] + bhn));
        const float hp = (h0 && orow < rows) ? h0[orow * ldh0 + c] : 0.f;
        hn[ct][q] = (1.0f - z) * n + z * hp;
        if (orow < rows) h_new[orow * C + c] = hn[ct][q];
      }
      __builtin_amdgcn_sched_barrier(0);  // one column tile's gates live at a time
    }
    for (int o = 0; o < n_out; ++o) {
      float wo[4];
#pragma unroll
      for (int ct = 0; ct < 4; ++ct) wo[ct] = w_out[o * C + 16 * ct + rl];
      const float bo = b_out ? b_out[o] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        float p = 0.f;
#pragma unroll
        for (int ct = 0; ct < 4; ++ct) p = fmaf(wo[ct], hn[ct][q], p);
        p = sum16(p);
        const int64_t orow = t * 16 + 4 * g + q;
        if (rl == 0 && orow < rows) out[orow * n_out + o] = p + bo;
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Training: the backward of the head (autograd of tgn.py:108-111 at
// loss.backward(), train.py:142), given dL/dout [rows, O] and (nullable)
// dL/dh_new [rows, C]:
//   dh' = dout W_out + dh_new
//   dn = dh' (1 - z), dz = dh' (h0 - n)          (h' = (1 - z) n + z h0)
//   dan = dn (1 - n^2), daz = dz z (1 - z), dar = dan (W_hn h0 + b_hn) r (1 - r)
//   gi = [dar | daz | dan]  (d of the x-side pre-activations: W_ih, b_ih, x)
//   gh = [dar | daz | dan r]  (h-side: W_hh, b_hh, h0)
//   grad_h = gi W_ih,  grad_h0 = gh W_hh + dh' z
// k_gru_head_bwd recomputes the gates exactly as k_gru_head does (same fp32
// MFMA products), writes gi / gh rows for the weight gradients (gfd_atb) and
// does both row GEMMs from a per-wave LDS tile of gi.  W_ih / W_hh are staged
// in LDS in their natural [3C][C] layout (pitch C + 4): read transposed for
// the gates, as they are for grad_h.
constexpr int kBW = 4;          // waves per block
constexpr int kWP = C + 4;      // LDS pitch of a W row (floats)
constexpr int kTP = kG + 4;     // LDS pitch of a gi tile row (floats)

size_t gru_bwd_smem(bool h0) {
  return sizeof(float) * (size_t(kG) * kWP * (h0 ? 2 : 1) + size_t(kBW) * 16 * kTP);
}

// gate column tile ct of rows (A layout of the forward: a[s][u] = row features
// 16 s + 4 g + u) against a natural-layout W in LDS
__device__ __forceinline__ f32x4 gate_tile(const f32x4 (&a)[4], const float* __restrict__ Wn,
                                           int ct, int rl, int g) {
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const f32x4 b = *reinterpret_cast<const f32x4*>(Wn + (16 * ct + rl) * kWP + 16 * s + 4 * g);
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s][u], b[u], acc, 0, 0, 0);
  }
  return acc;
}

// out tile nt of T[16 x 3C] (LDS, pitch kTP) . Wn[3C x C] (natural layout)
__device__ __forceinline__ f32x4 rowgemm_tile(const float* __restrict__ T,
                                              const float* __restrict__ Wn, int nt, int rl, int g,
                                              f32x4 acc) {
#pragma unroll 4
  for (int s = 0; s < kG / 16; ++s) {
    const f32x4 a = *reinterpret_cast<const f32x4*>(T + rl * kTP + 16 * s + 4 * g);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float b = Wn[(16 * s + 4 * g + u) * kWP + 16 * nt + rl];
      acc = __builtin_amdgcn_mfma_f32_16x16x4f32(a[u], b, acc, 0, 0, 0);
    }
  }
  return acc;
}

template <bool HAS_H0>
__global__ void __launch_bounds__(kBW * 64) k_gru_head_bwd(
    const float* __restrict__ h, int64_t ldh, int64_t rows, const float* __restrict__ w_ih,
    const float* __restrict__ b_ih, const float* __restrict__ w_hh, const float* __restrict__ b_hh,
    const float* __restrict__ h0, int64_t ldh0, const float* __restrict__ w_out, int n_out,
    const float* __restrict__ g_out, const float* __restrict__ g_hnew, float* __restrict__ grad_h,
    float* __restrict__ grad_h0, float* __restrict__ gi, float* __restrict__ gh) {
  extern __shared__ __attribute__((aligned(16))) char ssm[];
  float* Wi = reinterpret_cast<float*>(ssm);                 // [3C][kWP]
  float* Wh = Wi + kG * kWP;                                 // [3C][kWP] (HAS_H0)
  float* Tb = Wi + kG * kWP * (HAS_H0 ? 2 : 1);              // [kBW][16][kTP]
  for (int i = threadIdx.x; i < (HAS_H0 ? 2 : 1) * kG * (C / 4); i += blockDim.x) {
    const int which = i / (kG * (C / 4)), j = i % (kG * (C / 4));
    const int r = j / (C / 4), c4 = j % (C / 4);
    const float* W = which ? w_hh : w_ih;
    *reinterpret_cast<f32x4*>((which ? Wh : Wi) + r * kWP + 4 * c4) =
        *reinterpret_cast<const f32x4*>(W + r * C + 4 * c4);
  }
  __syncthreads();
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rl = lane & 15, g = lane >> 4;
  float* T = Tb + w * 16 * kTP;
  const int64_t wave = int64_t(blockIdx.x) * kBW + w;
  const int64_t nwave = int64_t(gridDim.x) * kBW;
  const int64_t tiles = (rows + 15) / 16;
  for (int64_t t = wave; t < tiles; t += nwave) {
    const int64_t row = t * 16 + rl;
    const int64_t rr = row < rows ? row : rows - 1;
    f32x4 a[4], a0[4];
#pragma unroll
    for (int s2 = 0; s2 < 4; ++s2) {
      a[s2] = *reinterpret_cast<const f32x4*>(h + rr * ldh + 16 * s2 + 4 * g);
      a0[s2] = HAS_H0 ? *reinterpret_cast<const f32x4*>(h0 + rr * ldh0 + 16 * s2 + 4 * g)
                      : f32x4{0.f, 0.f, 0.f, 0.f};
    }
    float dhz[4][4], ghn[4][4];
#pragma unroll
    for (int ct = 0; ct < 4; ++ct) {
      const f32x4 gr = gate_tile(a, Wi, ct, rl, g), gz = gate_tile(a, Wi, 4 + ct, rl, g),
                  gn = gate_tile(a, Wi, 8 + ct, rl, g);
      f32x4 hr = {0.f, 0.f, 0.f, 0.f}, hz = hr, hn = hr;
      if constexpr (HAS_H0) {
        hr = gate_tile(a0, Wh, ct, rl, g);
        hz = gate_tile(a0, Wh, 4 + ct, rl, g);
        hn = gate_tile(a0, Wh, 8 + ct, rl, g);
      }
      const int c = 16 * ct + rl;
      const float bir = b_ih ? b_ih[c] : 0.f, biz = b_ih ? b_ih[C + c] : 0.f,
                  bin = b_ih ? b_ih[2 * C + c] : 0.f;
      const float bhr = b_hh ? b_hh[c] : 0.f, bhz = b_hh ? b_hh[C + c] : 0.f,
                  bhn = b_hh ? b_hh[2 * C + c] : 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int rloc = 4 * g + q;
        const int64_t orow = t * 16 + rloc;
        const bool ok = orow < rows;
        const int64_t ro = ok ? orow : rows - 1;
        const float r = sigmoidf(gr[q] + bir + hr[q] + bhr);
        const float z = sigmoidf(gz[q] + biz + hz[q] + bhz);
        const float hnp = hn[q] + bhn;
        const float n = tanh_fast(gn[q] + bin + r * hnp);
        const float hp = HAS_H0 ? h0[ro * ldh0 + c] : 0.f;
        float dh = g_hnew ? g_hnew[ro * C + c] : 0.f;
        for (int o = 0; o < n_out; ++o) dh = fmaf(g_out[ro * n_out + o], w_out[o * C + c], dh);
        if (!ok) dh = 0.f;                       // rows past the end add nothing
        const float dan = dh * (1.0f - z) * (1.0f - n * n);
        const float daz = dh * (hp - n) * z * (1.0f - z);
        const float dar = dan * hnp * r * (1.0f - r);
        T[rloc * kTP + c] = dar;
        T[rloc * kTP + C + c] = daz;
        T[rloc * kTP + 2 * C + c] = dan;
        ghn[ct][q] = dan * r;
        dhz[ct][q] = dh * z;
        if (ok) {
          float* gir = gi + orow * kG;
          float* ghr = gh + orow * kG;
          gir[c] = dar; gir[C + c] = daz; gir[2 * C + c] = dan;
          ghr[c] = dar; ghr[C + c] = daz; ghr[2 * C + c] = dan * r;
        }
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    // grad_h = gi W_ih  (the tile is this wave's own: LDS ops retire in order)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const f32x4 acc = rowgemm_tile(T, Wi, nt, rl, g, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t orow = t * 16 + 4 * g + q;
        if (orow < rows) grad_h[orow * C + 16 * nt + rl] = acc[q];
      }
    }
    if constexpr (HAS_H0) {
      // grad_h0 = gh W_hh + dh' z  (gh = gi with the n gate times r)
#pragma unroll
      for (int ct = 0; ct < 4; ++ct)
#pragma unroll
        for (int q = 0; q < 4; ++q) T[(4 * g + q) * kTP + 2 * C + 16 * ct + rl] = ghn[ct][q];
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) {
        const f32x4 acc = rowgemm_tile(T, Wh, nt, rl, g,
                                       f32x4{dhz[nt][0], dhz[nt][1], dhz[nt][2], dhz[nt][3]});
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int64_t orow = t * 16 + 4 * g + q;
          if (orow < rows) grad_h0[orow * C + 16 * nt + rl] = acc[q];
        }
      }
    }
  }
}

// ---------------------------------------------------------------------------
// Weight gradients of a row-wise linear map (the GRUCell / Linear weight and
// bias gradients, sums over all rows): out[m][n] = sum_r A[r][m] B[r][n],
// colsum[m] = sum_r A[r][m], for m < M <= 192 and n < 64, in fp32 MFMA
// (16x16x4: exact products).  Split over S row slabs (block = 4 waves, wave w
// = output columns 16 w .. 16 w + 15, all m tiles; wave 0 also the column sums
// against a ones operand), then summed over the slabs in a fixed order:
// deterministic.
constexpr int kAtbMaxM = 192;
constexpr int kAtbSlabs = 256;

__global__ void __launch_bounds__(256) k_atb(const float* __restrict__ A, int64_t lda, int M,
                                              const float* __restrict__ B, int64_t ldb,
                                              int64_t rows, int64_t kps, float* __restrict__ part) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int rl = lane & 15, g = lane >> 4;
  const int MT = (M + 15) / 16;
  const int64_t r0 = int64_t(blockIdx.x) * kps, r1 = min(rows, r0 + kps);
  f32x4 acc[kAtbMaxM / 16], bac[kAtbMaxM / 16];
#pragma unroll
  for (int mt = 0; mt < kAtbMaxM / 16; ++mt) acc[mt] = bac[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int64_t k0 = r0; k0 < r1; k0 += 4) {
    const int64_t r = k0 + g;
    const bool ok = r < r1;
    const float b = ok ? B[r * ldb + 16 * w + rl] : 0.f;
#pragma unroll
    for (int mt = 0; mt < kAtbMaxM / 16; ++mt) {
      if (mt < MT) {
        const int m = 16 * mt + rl;
        const float av = (ok && m < M) ? A[r * lda + m] : 0.f;
        acc[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, b, acc[mt], 0, 0, 0);
        if (w == 0) bac[mt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, 1.0f, bac[mt], 0, 0, 0);
      }
    }
  }
  float* pr = part + int64_t(blockIdx.x) * (kAtbMaxM * C + kAtbMaxM);
#pragma unroll
  for (int mt = 0; mt < kAtbMaxM / 16; ++mt) {
    if (mt >= MT) continue;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int m = 16 * mt + 4 * g + q;
      if (m < M) {
        pr[m * C + 16 * w + rl] = acc[mt][q];
        if (w == 0 && rl == 0) pr[kAtbMaxM * C + m] = bac[mt][q];
      }
    }
  }
}

__global__ void __launch_bounds__(256) k_atb_reduce(const float* __restrict__ part, int S, int M,
                                                     float* __restrict__ out,
                                                     float* __restrict__ colsum) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int nw = M * C;
  if (i >= nw + M) return;
  const int off = i < nw ? i : kAtbMaxM * C + (i - nw);
  float v = 0.f;
  for (int s2 = 0; s2 < S; ++s2) v += part[int64_t(s2) * (kAtbMaxM * C + kAtbMaxM) + off];
  if (i < nw) out[i] = v;
  else if (colsum) colsum[i - nw] = v;
}

}  // namespace

extern "C" {

gfd_status gfd_gru_head_bwd(const float* h, int64_t rows, int channels, int64_t h_stride,
                            const float* w_ih, const float* b_ih, const float* w_hh,
                            const float* b_hh, const float* h0, int64_t h0_stride,
                            const float* w_out, int out_channels, const float* grad_out,
                            const float* grad_hnew, float* grad_h, float* grad_h0,
                            float* gates_i, float* gates_h, gfd_stream_t stream_) {
  if (channels != C) return GFD_ERR_UNSUPPORTED;
  if (rows < 0 || out_channels < 0 || out_channels > 64) return GFD_ERR_ARGUMENT;
  if (rows == 0) return GFD_OK;
  if (!h || !w_ih || !w_hh || !grad_h || !gates_i || !gates_h ||
      (out_channels > 0 && (!w_out || !grad_out)) || (h0 && !grad_h0))
    return GFD_ERR_ARGUMENT;
  if (h_stride < C || h_stride % 4 || (h0 && (h0_stride < C || h0_stride % 4)))
    return GFD_ERR_ARGUMENT;  // 16-B row loads
  if (reinterpret_cast<uintptr_t>(h) % 16 || (h0 && reinterpret_cast<uintptr_t>(h0) % 16) ||
      reinterpret_cast<uintptr_t>(w_ih) % 16 || reinterpret_cast<uintptr_t>(w_hh) % 16)
    return GFD_ERR_ARGUMENT;
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  const size_t lds = gru_bwd_smem(h0 != nullptr);
  auto kern = h0 ? &k_gru_head_bwd<true> : &k_gru_head_bwd<false>;
  if (!ensure_lds(reinterpret_cast<const void*>(kern), lds)) return GFD_ERR_HIP;
  const int64_t tiles = (rows + 15) / 16;
  int64_t nb = (tiles + kBW - 1) / kBW;
  const int64_t cap = int64_t(cu_count()) * 2;
  if (nb > cap) nb = cap;
  kern<<<int(nb), kBW * 64, lds, stream>>>(h, h_stride, rows, w_ih, b_ih, w_hh, b_hh, h0,
                                           h0_stride, w_out, out_channels, grad_out, grad_hnew,
                                           grad_h, grad_h0, gates_i, gates_h);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

size_t gfd_atb_workspace_size(int64_t rows, int m) {
  (void)rows;
  (void)m;
  return sizeof(float) * size_t(kAtbSlabs) * (kAtbMaxM * C + kAtbMaxM);
}

gfd_status gfd_atb(const float* A, int64_t lda, int m, const float* B, int64_t ldb, int64_t rows,
                   float* out, float* colsum, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  if (m < 1 || m > kAtbMaxM || rows < 0 || lda < m || ldb < C || !out) return GFD_ERR_ARGUMENT;
  if (rows > 0 && (!A || !B)) return GFD_ERR_ARGUMENT;
  if (!ws || ws_bytes < gfd_atb_workspace_size(rows, m)) return GFD_ERR_WORKSPACE;
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  float* part = static_cast<float*>(ws);
  int64_t S = (rows + 63) / 64;
  if (S > kAtbSlabs) S = kAtbSlabs;
  if (S < 1) S = 1;
  int64_t kps = (rows + S - 1) / S;
  kps = (kps + 3) / 4 * 4;
  if (rows > 0) {
    S = (rows + kps - 1) / kps;
    k_atb<<<unsigned(S), 256, 0, stream>>>(A, lda, m, B, ldb, rows, kps, part);
    GFD_LAUNCH_CHECK();
  } else {
    GFD_HIP_CHECK(hipMemsetAsync(part, 0, sizeof(float) * (kAtbMaxM * C + kAtbMaxM), stream));
    S = 1;
  }
  const int n = m * C + m;
  k_atb_reduce<<<unsigned((n + 255) / 256), 256, 0, stream>>>(part, int(S), m, out, colsum);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

gfd_status gfd_gru_head(const float* h, int64_t rows, int channels, int64_t h_stride,
                        const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, const float* h0, int64_t h0_stride,
                        const float* w_out, const float* b_out, int out_channels, float* h_new,
                        float* out, gfd_stream_t stream_) {
  if (channels != C) return GFD_ERR_UNSUPPORTED;
  if (rows < 0 || out_channels < 0 || out_channels > 64) return GFD_ERR_ARGUMENT;
  if (rows == 0) return GFD_OK;
  if (!h || !w_ih || !h_new || (out_channels > 0 && (!w_out || !out))) return GFD_ERR_ARGUMENT;
  if (h0 && !w_hh) return GFD_ERR_ARGUMENT;
  if (h_stride < C || h_stride % 4 || (h0 && (h0_stride < C || h0_stride % 4)))
    return GFD_ERR_ARGUMENT;  // 16-B row loads
  if (reinterpret_cast<uintptr_t>(h) % 16 || (h0 && reinterpret_cast<uintptr_t>(h0) % 16) ||
      reinterpret_cast<uintptr_t>(w_ih) % 16 || (w_hh && reinterpret_cast<uintptr_t>(w_hh) % 16))
    return GFD_ERR_ARGUMENT;
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  const size_t lds = sizeof(f32x4) * 12 * 4 * 64 * (h0 ? 2 : 1);
  if (!ensure_lds(reinterpret_cast<const void*>(&k_gru_head), lds)) return GFD_ERR_HIP;
  const int64_t tiles = (rows + 15) / 16;
  int64_t nb = (tiles + kHW - 1) / kHW;
  const int64_t cap = int64_t(cu_count()) * 2;
  if (nb > cap) nb = cap;
  k_gru_head<<<int(nb), kHW * 64, lds, stream>>>(h, h_stride, rows, w_ih, b_ih, w_hh, b_hh, h0,
                                                  h0_stride, w_out, b_out, out_channels, h_new,
                                                  out);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

}  // extern "C"
