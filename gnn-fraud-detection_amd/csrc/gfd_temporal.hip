// gfd_temporal.hip -- per-time-step snapshot extraction for config C3
// (SURVEY.md §8f rank 4): the reference's create_temporal_subgraph
// (/root/reference/src/data/dataset.py:198-240), which create_temporal_dataloaders
// (dataloader.py:99-135) calls once per time step with an O(E) Python loop,
// done for EVERY step in one pass on the device.
//
// Semantics (the reference's, per step t): the nodes whose time step is t in
// ascending id order, relabelled 0..n_t-1; the edges whose two endpoints are
// both in step t, in their original order, relabelled.  (The reference's loop
// tests `src in idx_mapping` with a 0-d tensor against int keys, which hashes
// by identity and keeps no edge at all; this implements the documented intent.)
//
//   node keys   step index s = time_step - t_first (S for nodes outside the range)
//   radix sort  (key, node id) pairs, stable  -> node_perm, node_pos = inverse
//   step_ptr    lower bounds of 0..S in the sorted keys
//   edge keys   s if both endpoints are in step s, else S (dropped)
//   radix sort  (key, edge id), stable -> edges grouped by step, original order
//   edge_ptr    lower bounds; kept edges written with global and local ids
#include <rocprim/device/device_radix_sort.hpp>

#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int kTB = 256;

inline int grid_of(int64_t n, int64_t cap = 65536) {
  int64_t g = (n + kTB - 1) / kTB;
  return int(g < 1 ? 1 : (g < cap ? g : cap));
}

inline int bits_of(int64_t v) {  // bits for values in [0, v]
  int b = 1;
  while ((int64_t(1) << b) <= v) ++b;
  return b;
}

__global__ void k_node_keys(const int64_t* __restrict__ ts, int64_t N, int64_t t_first, int S,
                            uint32_t* __restrict__ key, int32_t* __restrict__ val) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < N;
       i += int64_t(gridDim.x) * blockDim.x) {
    const int64_t s = ts[i] - t_first;
    key[i] = (s >= 0 && s < S) ? uint32_t(s) : uint32_t(S);
    val[i] = int32_t(i);
  }
}

__global__ void k_node_pos(const int32_t* __restrict__ perm, int64_t N, int32_t* __restrict__ pos) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < N;
       k += int64_t(gridDim.x) * blockDim.x)
    pos[perm[k]] = int32_t(k);
}

// ptr[s] = first position of key >= s in the sorted keys, s = 0..S
__global__ void k_lower_bounds(const uint32_t* __restrict__ skey, int64_t n, int S,
                               int64_t* __restrict__ ptr) {
  const int s = blockIdx.x * blockDim.x + threadIdx.x;
  if (s > S) return;
  int64_t lo = 0, hi = n;
  while (lo < hi) {
    const int64_t mid = (lo + hi) >> 1;
    if (skey[mid] < uint32_t(s)) lo = mid + 1; else hi = mid;
  }
  ptr[s] = lo;
}

__global__ void k_edge_keys(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                            const uint32_t* __restrict__ nkey, int S, uint32_t* __restrict__ key,
                            int32_t* __restrict__ val, int32_t* __restrict__ err) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < E;
       e += int64_t(gridDim.x) * blockDim.x) {
    const int64_t a = ei[e], b = ei[E + e];
    val[e] = int32_t(e);
    if (a < 0 || a >= N || b < 0 || b >= N) {
      atomicOr(err, 1);
      key[e] = uint32_t(S);
      continue;
    }
    const uint32_t ka = nkey[a], kb = nkey[b];
    key[e] = (ka == kb && ka < uint32_t(S)) ? ka : uint32_t(S);
  }
}

__global__ void k_edge_write(const int64_t* __restrict__ ei, int64_t E,
                             const uint32_t* __restrict__ skey, const int32_t* __restrict__ sval,
                             int S, const int32_t* __restrict__ pos,
                             const int64_t* __restrict__ step_ptr, int64_t* __restrict__ sub,
                             int64_t* __restrict__ sub_local) {
  for (int64_t k = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; k < E;
       k += int64_t(gridDim.x) * blockDim.x) {
    const uint32_t s = skey[k];
    if (s >= uint32_t(S)) continue;  // dropped edges sort last
    const int64_t e = sval[k];
    const int64_t a = ei[e], b = ei[E + e];
    sub[k] = a;
    sub[E + k] = b;
    if (sub_local) {
      sub_local[k] = pos[a] - step_ptr[s];
      sub_local[E + k] = pos[b] - step_ptr[s];
    }
  }
}

size_t sort_tmp_bytes(int64_t n, int bits) {
  size_t t = 0;
  (void)rocprim::radix_sort_pairs(nullptr, t, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (int32_t*)nullptr, (int32_t*)nullptr, size_t(n > 0 ? n : 1), 0,
                                  bits);
  return t;
}

size_t temporal_layout(int64_t N, int64_t E, int S, size_t* tn, size_t* te) {
  const int bits = bits_of(S);
  *tn = sort_tmp_bytes(N, bits);
  *te = sort_tmp_bytes(E, bits);
  Sizer s;
  s.take<uint32_t>(N); s.take<uint32_t>(N); s.take<int32_t>(N);       // node keys, sorted, ids
  s.take<uint32_t>(E); s.take<uint32_t>(E); s.take<int32_t>(E); s.take<int32_t>(E);
  s.take<int32_t>(4);
  s.take<char>(*tn); s.take<char>(*te);
  return s.off;
}

}  // namespace

extern "C" {

size_t gfd_temporal_workspace_size(int64_t num_nodes, int64_t num_edges, int32_t num_steps) {
  if (num_nodes <= 0 || num_edges < 0 || num_steps <= 0) return 0;
  size_t a, b;
  return temporal_layout(num_nodes, num_edges, num_steps, &a, &b);
}

gfd_status gfd_temporal_snapshots(const int64_t* time_step, int64_t N, const int64_t* edge_index,
                                  int64_t E, int64_t t_first, int32_t S, int32_t* node_perm,
                                  int32_t* node_pos, int64_t* step_ptr, int64_t* sub_edge_index,
                                  int64_t* sub_edge_local, int64_t* edge_ptr, void* ws,
                                  size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (N <= 0 || E < 0 || S <= 0 || !time_step || (E > 0 && (!edge_index || !sub_edge_index)) ||
      !node_perm || !node_pos || !step_ptr || !edge_ptr)
    return GFD_ERR_ARGUMENT;
  if (N >= (int64_t(1) << 31) || E >= (int64_t(1) << 31) || S >= (1 << 30))
    return GFD_ERR_UNSUPPORTED;
  size_t tn, te;
  if (!ws || ws_bytes < temporal_layout(N, E, S, &tn, &te)) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  uint32_t* nkey = c.take<uint32_t>(N);
  uint32_t* nkey_s = c.take<uint32_t>(N);
  int32_t* nid = c.take<int32_t>(N);
  uint32_t* ekey = c.take<uint32_t>(E);
  uint32_t* ekey_s = c.take<uint32_t>(E);
  int32_t* eid = c.take<int32_t>(E);
  int32_t* eid_s = c.take<int32_t>(E);
  int32_t* err = c.take<int32_t>(4);
  void* tmp_n = c.take<char>(tn);
  void* tmp_e = c.take<char>(te);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  const int bits = bits_of(S);
  GFD_HIP_CHECK(hipMemsetAsync(err, 0, sizeof(int32_t) * 4, stream));
  k_node_keys<<<grid_of(N), kTB, 0, stream>>>(time_step, N, t_first, S, nkey, nid);
  GFD_LAUNCH_CHECK();
  size_t t = tn;
  if (rocprim::radix_sort_pairs(tmp_n, t, nkey, nkey_s, nid, node_perm, size_t(N), 0, bits,
                                stream) != hipSuccess)
    return GFD_ERR_HIP;
  k_node_pos<<<grid_of(N), kTB, 0, stream>>>(node_perm, N, node_pos);
  GFD_LAUNCH_CHECK();
  k_lower_bounds<<<(S + 1 + kTB - 1) / kTB, kTB, 0, stream>>>(nkey_s, N, S, step_ptr);
  GFD_LAUNCH_CHECK();
  if (E > 0) {
    k_edge_keys<<<grid_of(E), kTB, 0, stream>>>(edge_index, E, N, nkey, S, ekey, eid, err);
    GFD_LAUNCH_CHECK();
    t = te;
    if (rocprim::radix_sort_pairs(tmp_e, t, ekey, ekey_s, eid, eid_s, size_t(E), 0, bits,
                                  stream) != hipSuccess)
      return GFD_ERR_HIP;
    k_lower_bounds<<<(S + 1 + kTB - 1) / kTB, kTB, 0, stream>>>(ekey_s, E, S, edge_ptr);
    GFD_LAUNCH_CHECK();
    k_edge_write<<<grid_of(E), kTB, 0, stream>>>(edge_index, E, ekey_s, eid_s, S, node_pos,
                                                 step_ptr, sub_edge_index, sub_edge_local);
    GFD_LAUNCH_CHECK();
  } else {
    GFD_HIP_CHECK(hipMemsetAsync(edge_ptr, 0, sizeof(int64_t) * (S + 1), stream));
  }
  int32_t herr = 0;
  GFD_HIP_CHECK(hipMemcpyAsync(&herr, err, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
  GFD_HIP_CHECK(hipStreamSynchronize(stream));
  return herr ? GFD_ERR_INDEX : GFD_OK;
}

}  // extern "C"
