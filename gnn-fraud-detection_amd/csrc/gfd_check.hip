// gfd_check.hip -- device validation of the index arrays (the bounds-checked
// diagnostic build, gfd_check.h).  Compiled to a no-op without GFD_CHECKED.
#include <mutex>

#include "gfd_check.h"

namespace gfd {

#ifdef GFD_CHECKED
__device__ CheckRecord g_check;

namespace {

constexpr int kCB = 256;

__global__ void k_check_rows(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                             int64_t n, int64_t N) {
  const int64_t i = blockIdx.x * int64_t(kCB) + threadIdx.x;
  if (i > n) return;
  if (i == 0) GFD_DCHECK("rowptr[0] (range start)", 0, rowptr[0], 0, rowptr[n] + 1);
  if (i < n) {
    const int64_t e0 = rowptr[i], e1 = rowptr[i + 1];
    GFD_DCHECK("rowptr (monotone, <= rowptr[n])", i + 1, e1, e0, int64_t(rowptr[n]) + 1);
    for (int64_t e = e0; e < e1; ++e) GFD_DCHECK("col", e, col[e], 0, N);
  }
}

__global__ void k_check_slots(const int32_t* __restrict__ rowptr, const int4* __restrict__ desc,
                              const int32_t* __restrict__ cols8, int64_t n, int64_t N,
                              int64_t num_hubs) {
  const int64_t s = blockIdx.x * int64_t(kCB) + threadIdx.x;
  if (s >= n) return;
  const int4 d = desc[s];
  GFD_DCHECK("slot_desc.row", s, d.x, 0, n);
  GFD_DCHECK("slot_desc.e_begin", s, d.y, rowptr[d.x], rowptr[d.x] + 1);
  GFD_DCHECK("slot_desc.e_end", s, d.z, rowptr[d.x + 1], rowptr[d.x + 1] + 1);
  GFD_DCHECK("slot_desc.hub_rank", s, d.w, -1, num_hubs);
  if (cols8)
    for (int k = 0; k < 8; ++k) GFD_DCHECK("slot_cols", 8 * s + k, cols8[8 * s + k], 0, N);
}

__global__ void k_check_chunks(const int4* __restrict__ ck, int64_t nc,
                               const int32_t* __restrict__ rowptr, int64_t n, int64_t num_hubs,
                               const int32_t* __restrict__ hub_dst) {
  const int64_t c = blockIdx.x * int64_t(kCB) + threadIdx.x;
  if (c >= nc) return;
  const int4 k = ck[c];
  GFD_DCHECK("hub_chunk.hub", c, k.x, 0, num_hubs);
  GFD_DCHECK("hub_chunk.dst", c, k.w, 0, n);
  GFD_DCHECK("hub_dst", k.x, hub_dst[k.x], k.w, k.w + 1);
  GFD_DCHECK("hub_chunk.e_begin", c, k.y, rowptr[k.w], rowptr[k.w + 1]);
  GFD_DCHECK("hub_chunk.e_end", c, k.z, k.y + 1, rowptr[k.w + 1] + 1);
}

__global__ void k_check_csc(const int32_t* __restrict__ colptr, const int32_t* __restrict__ dst,
                            const int32_t* __restrict__ eid, int64_t N, int64_t M) {
  const int64_t j = blockIdx.x * int64_t(kCB) + threadIdx.x;
  if (j >= N) return;
  const int64_t p0 = colptr[j], p1 = colptr[j + 1];
  GFD_DCHECK("colptr (monotone)", j + 1, p1, p0, M + 1);
  for (int64_t p = p0; p < p1; ++p) {
    GFD_DCHECK("csc_dst", p, dst[p], 0, N);
    GFD_DCHECK("csc_eid", p, eid[p], 0, M);
  }
}

unsigned blocks(int64_t n) { return unsigned((n + kCB - 1) / kCB); }

}  // namespace
#endif

gfd_status check_graph(const int32_t* rowptr, const int32_t* col, int64_t num_dst, int64_t N,
                       const gfd_plan* plan, const int32_t* colptr, const int32_t* csc_dst,
                       const int32_t* csc_eid, int64_t num_messages, hipStream_t stream) {
#ifdef GFD_CHECKED
  // one record per device: calls on other streams (per-rank threads, the
  // sampler's stream) would clear or read each other's -- the checked build
  // serialises check_graph across host threads
  static std::mutex mu;
  std::lock_guard<std::mutex> lock(mu);
  void* rec = nullptr;
  if (hipGetSymbolAddress(&rec, HIP_SYMBOL(g_check)) != hipSuccess) return GFD_ERR_HIP;
  if (hipMemsetAsync(rec, 0, sizeof(CheckRecord), stream) != hipSuccess) return GFD_ERR_HIP;
  if (num_dst > 0) {
    k_check_rows<<<blocks(num_dst + 1), kCB, 0, stream>>>(rowptr, col, num_dst, N);
    GFD_LAUNCH_CHECK();
  }
  if (plan && plan->slot_desc && num_dst > 0) {
    k_check_slots<<<blocks(num_dst), kCB, 0, stream>>>(
        rowptr, reinterpret_cast<const int4*>(plan->slot_desc), plan->slot_cols, num_dst, N,
        plan->num_hubs);
    GFD_LAUNCH_CHECK();
  }
  if (plan && plan->num_hubs > 0 && plan->num_chunks > 0) {
    k_check_chunks<<<blocks(plan->num_chunks), kCB, 0, stream>>>(
        reinterpret_cast<const int4*>(plan->hub_chunk), plan->num_chunks, rowptr, num_dst,
        plan->num_hubs, plan->hub_dst);
    GFD_LAUNCH_CHECK();
  }
  if (colptr && csc_dst && csc_eid) {
    k_check_csc<<<blocks(N), kCB, 0, stream>>>(colptr, csc_dst, csc_eid, N, num_messages);
    GFD_LAUNCH_CHECK();
  }
  CheckRecord host{};
  if (hipMemcpyAsync(&host, rec, sizeof(host), hipMemcpyDeviceToHost, stream) != hipSuccess ||
      hipStreamSynchronize(stream) != hipSuccess)
    return GFD_ERR_HIP;
  if (host.flag) return GFD_ERR_INDEX;
#else
  (void)rowptr; (void)col; (void)num_dst; (void)N; (void)plan; (void)colptr; (void)csc_dst;
  (void)csc_eid; (void)num_messages; (void)stream;
#endif
  return GFD_OK;
}

}  // namespace gfd
