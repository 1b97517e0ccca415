// gfd_hub.hip -- hub destinations (more than `hub_threshold` messages): the
// segment softmax and aggregation of PyG GATConv (utils.softmax + propagate,
// inside /root/reference/src/models/gat.py:80) split into chunks so no wave
// runs a whole power-law hub.
//
//   k_hub_partial  one wave per chunk: online softmax over the chunk, partial
//                  (max, sum, unnormalised z[8][Fp]) to the workspace
//   k_hub_fin      per hub: global (max, sum) per head over its chunks, then the
//                  merged, normalised z row (read by the tile kernels)
#include "gfd_fwd.h"

using namespace gfd;
using namespace gfd::fwd;

namespace {

// four waves per SIMD (<= 128 VGPRs at KF = 3), two batches of 8 rows in flight each;
// PAIR (bf16 rows, 128 < F <= 192, 4-B aligned rows): GFD_HUB_NBF_PAIR batches
// of 2-VGPR rows (aggregate_segment_bf16p)
#ifndef GFD_HUB_PAIR
#define GFD_HUB_PAIR 1
#endif
#ifndef GFD_HUB_NBF_PAIR
#define GFD_HUB_NBF_PAIR 3  // 4: the allocator spills (1.8k VGPRs at 128)
#endif
template <typename XT, int KF, bool PAIR>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(4))) k_hub_partial(
    const void* __restrict__ x, int F, int Fp, int64_t ldx, const int32_t* __restrict__ col,
    const float* __restrict__ s, int lds, const float* __restrict__ t, int ldt, float slope, float dp, uint64_t seed,
    const int4* __restrict__ chunks, int64_t num_chunks, float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t c = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  if (c >= num_chunks) return;
  const int4 ck = chunks[c];
  const float t_h = lrow(t, ck.w, ldt)[lane & 7];
  float acc[H][KF];
  SegState S;
  if constexpr (PAIR) {
    static_assert(KF == 3, "bf16 pairs: 128 < F <= 192");
    S = aggregate_segment_bf16p<GFD_HUB_NBF_PAIR>(x, ldx, F, col, ck.y, ck.z, s, lds, t_h, slope,
                                                  dp, seed, acc);
  } else {
    S = aggregate_segment<XT, KF>(x, ldx, F, col, ck.y, ck.z, s, lds, t_h, slope, dp, seed, acc);
  }
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
      const int f = PAIR ? seg_feat_pair(q, lane) : lane + 64 * q;
      if (f < Fp) pr[16 + hh * Fp + f] = acc[hh][q];
    }
}

// Hub finalisation, one wave per (hub, K slice of 256 values): global (max,
// sum) per head over the hub's chunk partials (lanes over chunks), then the
// slice of the merged, normalised z row (16-B loads).  Fp is a multiple of 8,
// so a 4-wide group never straddles heads.  Writes the backward's stats too.
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

template <typename XT, int KF>
gfd_status launch_hubs_t(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  const gfd_plan& p = a.plan;
  const int64_t blocks = (p.num_chunks + 3) / 4;
  // bf16 pairs: 4-B loads need every row start 4-B aligned
  const bool pair = GFD_HUB_PAIR && XT::kBytes == 2 && KF == 3 && a.F > 128 &&
                    reinterpret_cast<uintptr_t>(a.x) % 4 == 0 && a.ldx % 2 == 0;
  auto kern = pair ? &k_hub_partial<XT, KF, (XT::kBytes == 2 && KF == 3)>
                   : &k_hub_partial<XT, KF, false>;
  kern<<<int(blocks), 256, 0, stream>>>(
      a.x, a.F, L.Fp, a.ldx, a.col, a.s, a.lds, a.t, a.ldt, a.slope, a.dp, a.seed,
      reinterpret_cast<const int4*>(p.hub_chunk), p.num_chunks, a.part);
  GFD_LAUNCH_CHECK();
  const int slices = (L.KP / 4 + 63) / 64;
  k_hub_fin<<<unsigned((p.num_hubs * slices + 3) / 4), 256, 0, stream>>>(
      a.part, L.Fp, p.hub_chunk_ptr, p.hub_dst, p.num_hubs, slices, a.stats, a.zhub);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

template <typename XT>
gfd_status launch_hubs_x(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  switch (kf_for(a.F)) {
    case 1: return launch_hubs_t<XT, 1>(a, L, stream);
    case 2: return launch_hubs_t<XT, 2>(a, L, stream);
    case 3: return launch_hubs_t<XT, 3>(a, L, stream);
    case 4: return launch_hubs_t<XT, 4>(a, L, stream);
    default: return GFD_ERR_UNSUPPORTED;
  }
}

}  // namespace

namespace gfd {
namespace fwd {

gfd_status launch_hubs(const AggArgs& a, const PackLayout& L, hipStream_t stream) {
  if (a.plan.num_hubs <= 0) return GFD_OK;
  return a.xdt == GFD_DTYPE_BF16 ? launch_hubs_x<XBF16>(a, L, stream)
                                 : launch_hubs_x<XF32>(a, L, stream);
}

}  // namespace fwd
}  // namespace gfd
