// gfd_ingest.hip -- graph ingest on the device: the
// id -> index mapping and edge filtering of the reference's
// EllipticBitcoinDataset.process (/root/reference/src/data/dataset.py:75-129),
// which builds a Python dict of 203k transaction ids and walks every edge row
// and every class row with DataFrame.iterrows().
//
//   gfd_id_map_build   sort (id, index) pairs: the dict node_id_to_idx (:92)
//   gfd_id_map_lookup  binary search per query id (-1 when unknown): the
//                      `in node_id_to_idx` tests of :97 and :111
//   gfd_edges_from_ids edges whose two endpoints are known, original order
//                      (:95-101): a stable compaction (prefix sum of flags)
// Duplicate ids map to the LAST index (a dict comprehension keeps the last).
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int kIB = 256;

inline int igrid(int64_t n) {
  int64_t g = (n + kIB - 1) / kIB;
  return int(g < 1 ? 1 : (g < 65536 ? g : 65536));
}

__global__ void k_iota(int32_t* __restrict__ v, int64_t n) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    v[i] = int32_t(i);
}

// index of the LAST occurrence of q among the sorted keys (stable sort keeps
// equal ids in index order), -1 when absent
__device__ __forceinline__ int32_t lookup(const int64_t* __restrict__ keys,
                                          const int32_t* __restrict__ idx, int64_t n, int64_t q) {
  int64_t lo = 0, hi = n;  // first key > q
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (keys[mid] <= q) lo = mid + 1; else hi = mid;
  }
  return (lo > 0 && keys[lo - 1] == q) ? idx[lo - 1] : -1;
}

__global__ void k_lookup(const int64_t* __restrict__ keys, const int32_t* __restrict__ idx,
                         int64_t n, const int64_t* __restrict__ q, int64_t m,
                         int32_t* __restrict__ out) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < m;
       i += int64_t(gridDim.x) * blockDim.x)
    out[i] = lookup(keys, idx, n, q[i]);
}

__global__ void k_edge_flags(const int64_t* __restrict__ keys, const int32_t* __restrict__ idx,
                             int64_t n, const int64_t* __restrict__ src_ids,
                             const int64_t* __restrict__ dst_ids, int64_t E,
                             int32_t* __restrict__ s, int32_t* __restrict__ d,
                             int64_t* __restrict__ flag) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < E;
       e += int64_t(gridDim.x) * blockDim.x) {
    const int32_t a = lookup(keys, idx, n, src_ids[e]);
    const int32_t b = lookup(keys, idx, n, dst_ids[e]);
    s[e] = a;
    d[e] = b;
    flag[e] = (a >= 0 && b >= 0) ? 1 : 0;
  }
}

__global__ void k_edge_compact(const int32_t* __restrict__ s, const int32_t* __restrict__ d,
                               const int64_t* __restrict__ flag, const int64_t* __restrict__ pos,
                               int64_t E, int64_t* __restrict__ out, int64_t* __restrict__ count) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < E;
       e += int64_t(gridDim.x) * blockDim.x) {
    if (flag[e]) {
      out[pos[e]] = s[e];
      out[E + pos[e]] = d[e];
    }
    if (e == E - 1) *count = pos[e] + flag[e];
  }
}

size_t sort_bytes(int64_t n) {
  size_t t = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t, (int64_t*)nullptr, (int64_t*)nullptr,
                                  (int32_t*)nullptr, (int32_t*)nullptr, size_t(n > 0 ? n : 1));
  return t;
}

size_t scan_bytes(int64_t n) {
  size_t t = 0;
  (void)rocprim::exclusive_scan(nullptr, t, (const int64_t*)nullptr, (int64_t*)nullptr,
                                int64_t(0), size_t(n > 0 ? n : 1), rocprim::plus<int64_t>());
  return t;
}

}  // namespace

extern "C" {

size_t gfd_id_map_workspace_size(int64_t num_ids) {
  if (num_ids <= 0) return 0;
  Sizer s;
  s.take<int32_t>(num_ids);
  s.take<char>(sort_bytes(num_ids));
  return s.off;
}

gfd_status gfd_id_map_build(const int64_t* ids, int64_t n, int64_t* sorted_ids,
                            int32_t* sorted_idx, void* ws, size_t ws_bytes,
                            gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!ids || n <= 0 || !sorted_ids || !sorted_idx) return GFD_ERR_ARGUMENT;
  if (n >= (int64_t(1) << 31)) return GFD_ERR_UNSUPPORTED;
  const size_t st = sort_bytes(n);
  Carve c(ws, ws_bytes);
  int32_t* iota = c.take<int32_t>(n);
  void* tmp = c.take<char>(st);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  k_iota<<<igrid(n), kIB, 0, stream>>>(iota, n);
  GFD_LAUNCH_CHECK();
  size_t t = st;
  if (rocprim::radix_sort_pairs(tmp, t, ids, sorted_ids, iota, sorted_idx, size_t(n), 0,
                                int(8 * sizeof(int64_t)), stream) != hipSuccess)
    return GFD_ERR_HIP;
  return GFD_OK;
}

gfd_status gfd_id_map_lookup(const int64_t* sorted_ids, const int32_t* sorted_idx, int64_t n,
                             const int64_t* queries, int64_t num_queries, int32_t* out,
                             gfd_stream_t stream_) {
  if (!sorted_ids || !sorted_idx || n <= 0 || num_queries < 0 ||
      (num_queries > 0 && (!queries || !out)))
    return GFD_ERR_ARGUMENT;
  if (num_queries == 0) return GFD_OK;
  k_lookup<<<igrid(num_queries), kIB, 0, static_cast<hipStream_t>(stream_)>>>(
      sorted_ids, sorted_idx, n, queries, num_queries, out);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

size_t gfd_edges_from_ids_workspace_size(int64_t num_edges) {
  if (num_edges <= 0) return 0;
  Sizer s;
  s.take<int32_t>(num_edges); s.take<int32_t>(num_edges);
  s.take<int64_t>(num_edges); s.take<int64_t>(num_edges);
  s.take<char>(scan_bytes(num_edges));
  return s.off;
}

gfd_status gfd_edges_from_ids(const int64_t* sorted_ids, const int32_t* sorted_idx, int64_t n,
                              const int64_t* src_ids, const int64_t* dst_ids, int64_t E,
                              int64_t* edge_index, int64_t* num_kept, void* ws, size_t ws_bytes,
                              gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!sorted_ids || !sorted_idx || n <= 0 || E < 0 || !num_kept) return GFD_ERR_ARGUMENT;
  if (E == 0) return hipMemsetAsync(num_kept, 0, sizeof(int64_t), stream) == hipSuccess
                         ? GFD_OK : GFD_ERR_HIP;
  if (!src_ids || !dst_ids || !edge_index) return GFD_ERR_ARGUMENT;
  const size_t sb = scan_bytes(E);
  Carve c(ws, ws_bytes);
  int32_t* s = c.take<int32_t>(E);
  int32_t* d = c.take<int32_t>(E);
  int64_t* flag = c.take<int64_t>(E);
  int64_t* pos = c.take<int64_t>(E);
  void* tmp = c.take<char>(sb);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  k_edge_flags<<<igrid(E), kIB, 0, stream>>>(sorted_ids, sorted_idx, n, src_ids, dst_ids, E, s, d,
                                             flag);
  GFD_LAUNCH_CHECK();
  size_t t = sb;
  if (rocprim::exclusive_scan(tmp, t, flag, pos, int64_t(0), size_t(E), rocprim::plus<int64_t>(),
                              stream) != hipSuccess)
    return GFD_ERR_HIP;
  k_edge_compact<<<igrid(E), kIB, 0, stream>>>(s, d, flag, pos, E, edge_index, num_kept);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

}  // extern "C"
