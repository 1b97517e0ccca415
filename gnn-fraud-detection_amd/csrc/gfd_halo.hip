// gfd_halo.hip -- row gather / scatter of the sparse halo exchange between
// destination shards (gfd.dist.HaloPlan).  The north star's
// "RCCL all-gather of halo features" moves every node's source logits s_j
// (32 B) to every rank; a rank's in-edges reference only ~22 % of the other
// ranks' nodes at C4 over 8 ranks, so the shard exchange sends each peer just
// the rows it reads:
//   send: buf[i] = table[send_rows[i]]   (the rank's own rows a peer needs)
//   RCCL all_to_all_single(recv, buf)    (host side, uneven splits)
//   recv: table[recv_rows[i]] = recv[i]  (at the node rows the kernels read)
// One kernel for both directions: dst[dst_rows[i]] = src[src_rows[i]] (either
// index list may be NULL = identity).  HBM-bound, 2 x 4 x cols bytes per row
// plus 4-8 B of indices.
#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int kRB = 256;

// V floats per access (4: one 16-B load / store, 1: 4 B); PER accesses per
// row when known at compile time (2: the 8-float logits rows, 18: the 72-float
// hidden rows), else the runtime ``per``.  Element counts below 2^31 (every
// exchange here): 32-bit index arithmetic.
template <int V, int PER>
__global__ void __launch_bounds__(kRB) k_rows_copy(const float* __restrict__ src, int64_t lds,
                                                   const int32_t* __restrict__ sidx,
                                                   float* __restrict__ dst, int64_t ldd,
                                                   const int32_t* __restrict__ didx, int64_t n,
                                                   int per_rt) {
  const uint32_t per = PER > 0 ? uint32_t(PER) : uint32_t(per_rt);
  const uint32_t total = uint32_t(n) * per;
  const uint32_t step = gridDim.x * kRB;
  for (uint32_t i = blockIdx.x * kRB + threadIdx.x; i < total; i += step) {
    const uint32_t r = i / per;
    const int c = int(i - r * per) * V;
    const int64_t rs = sidx ? int64_t(sidx[r]) : r;
    const int64_t rd = didx ? int64_t(didx[r]) : r;
    if constexpr (V == 4) {
      *reinterpret_cast<float4*>(dst + rd * ldd + c) =
          *reinterpret_cast<const float4*>(src + rs * lds + c);
    } else {
      dst[rd * ldd + c] = src[rs * lds + c];
    }
  }
}

}  // namespace

extern "C" {

gfd_status gfd_rows_copy(const float* src, int64_t src_stride, const int32_t* src_rows,
                         float* dst, int64_t dst_stride, const int32_t* dst_rows, int64_t n,
                         int cols, gfd_stream_t stream_) {
  if (n < 0 || cols < 1 || src_stride < cols || dst_stride < cols) return GFD_ERR_ARGUMENT;
  if (n == 0) return GFD_OK;
  if (!src || !dst) return GFD_ERR_ARGUMENT;
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  const bool v4 = cols % 4 == 0 && src_stride % 4 == 0 && dst_stride % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(src) % 16 == 0 &&
                  reinterpret_cast<uintptr_t>(dst) % 16 == 0;
  const int per = v4 ? cols / 4 : cols;
  const int64_t total = n * per;
  if (total >= (int64_t(1) << 31)) return GFD_ERR_UNSUPPORTED;
  int64_t grid = (total + kRB - 1) / kRB;
  if (grid > 8192) grid = 8192;  // grid-stride beyond 32 blocks per CU
#define GFD_RC(V, PER)                                                                       \
  k_rows_copy<V, PER><<<int(grid), kRB, 0, stream>>>(src, src_stride, src_rows, dst, dst_stride, \
                                                     dst_rows, n, per)
  if (v4 && per == 2) GFD_RC(4, 2);
  else if (v4 && per == 18) GFD_RC(4, 18);
  else if (v4) GFD_RC(4, 0);
  else GFD_RC(1, 0);
#undef GFD_RC
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

}  // extern "C"
