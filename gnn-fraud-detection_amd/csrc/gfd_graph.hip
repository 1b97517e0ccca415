// gfd_graph.hip -- COO -> destination-sorted CSR (PyG self-loop policy), its
// source-sorted (CSC) view, and the hub plan.  Replaces PyG GATConv's per-call
// remove_self_loops/add_self_loops and index bookkeeping (SURVEY.md §2 op 3).
// Built once per graph and cached by the caller; never on the timed path.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n, int block = kBlock, int64_t cap = 65536) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  return int(g < cap ? g : cap);
}

inline int bits_for(int64_t v) {  // bits needed to represent values in [0, v]
  int b = 1;
  while ((int64_t(1) << b) <= v) ++b;
  return b;
}

// key = dst (or N for a self loop, sorted last and dropped), val = src.
__global__ void k_coo_keys(const int64_t* __restrict__ ei, int64_t E, int64_t N,
                           uint32_t* __restrict__ key, int32_t* __restrict__ val,
                           int32_t* __restrict__ deg, int32_t* __restrict__ err) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < E;
       e += int64_t(gridDim.x) * blockDim.x) {
    int64_t s = ei[e], d = ei[E + e];
    bool bad = (s < 0) | (s >= N) | (d < 0) | (d >= N);
    if (bad) { atomicOr(err, 1); key[e] = uint32_t(N); val[e] = 0; continue; }
    if (s == d) { key[e] = uint32_t(N); val[e] = int32_t(s); continue; }
    key[e] = uint32_t(d);
    val[e] = int32_t(s);
    atomicAdd(&deg[d], 1);
  }
}

__global__ void k_plus_one(const int32_t* __restrict__ deg, int32_t* __restrict__ cnt, int64_t N) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= N;
       i += int64_t(gridDim.x) * blockDim.x)
    cnt[i] = i < N ? deg[i] + 1 : 0;
}

// Sorted (dst, src) pairs -> col; p-th kept pair with dst d lands at p + d
// (d self loops precede it).  Self loop of node i is the last entry of row i.
__global__ void k_fill_col(const uint32_t* __restrict__ skey, const int32_t* __restrict__ sval,
                           int64_t E, int64_t N, const int32_t* __restrict__ rowptr,
                           int32_t* __restrict__ col) {
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < E;
       p += int64_t(gridDim.x) * blockDim.x) {
    uint32_t d = skey[p];
    if (d < uint32_t(N)) col[p + d] = sval[p];
  }
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < N;
       i += int64_t(gridDim.x) * blockDim.x)
    col[rowptr[i + 1] - 1] = int32_t(i);
}

// CSR -> (key = src, val = CSR position); also counts messages per source.
__global__ void k_csr_keys(const int32_t* __restrict__ col, int64_t M, uint32_t* __restrict__ key,
                           int32_t* __restrict__ val, int32_t* __restrict__ cnt) {
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < M;
       e += int64_t(gridDim.x) * blockDim.x) {
    int32_t s = col[e];
    key[e] = uint32_t(s);
    val[e] = int32_t(e);
    atomicAdd(&cnt[s], 1);
  }
}

// row index of every CSR position (one wave per row keeps it coalesced).
__global__ void k_row_of(const int32_t* __restrict__ rowptr, int64_t N, int32_t* __restrict__ rowid) {
  int lane = threadIdx.x & 63;
  int64_t w = (blockIdx.x * int64_t(blockDim.x) + threadIdx.x) >> 6;
  int64_t nw = (int64_t(gridDim.x) * blockDim.x) >> 6;
  for (int64_t i = w; i < N; i += nw) {
    int32_t b = rowptr[i], e = rowptr[i + 1];
    for (int32_t p = b + lane; p < e; p += 64) rowid[p] = int32_t(i);
  }
}

__global__ void k_gather_dst(const int32_t* __restrict__ eid, const int32_t* __restrict__ rowid,
                             int64_t M, int32_t* __restrict__ dst) {
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < M;
       p += int64_t(gridDim.x) * blockDim.x)
    dst[p] = rowid[eid[p]];
}

// ---- hub plan ----
__global__ void k_hub_flags(const int32_t* __restrict__ rowptr, int64_t n, int32_t thr, int32_t chunk,
                            int32_t* __restrict__ is_hub, int32_t* __restrict__ nchunk) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i <= n;
       i += int64_t(gridDim.x) * blockDim.x) {
    if (i == n) { is_hub[i] = 0; nchunk[i] = 0; continue; }
    int32_t d = rowptr[i + 1] - rowptr[i];
    bool h = d > thr;
    is_hub[i] = h;
    nchunk[i] = h ? (d + chunk - 1) / chunk : 0;
  }
}

__global__ void k_hub_write(const int32_t* __restrict__ rowptr, int64_t n, int32_t thr, int32_t chunk,
                            const int32_t* __restrict__ hub_idx, const int32_t* __restrict__ chunk_off,
                            int32_t* __restrict__ hub_rank, int32_t* __restrict__ hub_chunk,
                            int32_t* __restrict__ hub_chunk_ptr, int32_t* __restrict__ hub_dst,
                            int64_t max_hubs, int64_t max_chunks) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    int32_t b = rowptr[i], e = rowptr[i + 1];
    if (e - b <= thr) { hub_rank[i] = -1; continue; }
    int32_t h = hub_idx[i];
    hub_rank[i] = h;
    if (h >= max_hubs) continue;
    hub_dst[h] = int32_t(i);
    int32_t c0 = chunk_off[i];
    hub_chunk_ptr[h] = c0;
    for (int32_t c = 0, p = b; p < e; ++c, p += chunk) {
      if (c0 + c >= max_chunks) break;
      int32_t* q = hub_chunk + 4 * int64_t(c0 + c);
      q[0] = h; q[1] = p; q[2] = min(p + chunk, e); q[3] = int32_t(i);
    }
  }
}

__global__ void k_hub_tail(const int32_t* __restrict__ hub_idx, const int32_t* __restrict__ chunk_off,
                           int64_t n, int32_t* __restrict__ hub_chunk_ptr, int64_t max_hubs,
                           int64_t* __restrict__ counts) {
  int32_t nh = hub_idx[n], nc = chunk_off[n];
  counts[0] = nh;
  counts[1] = nc;
  if (nh <= max_hubs && hub_chunk_ptr != nullptr) hub_chunk_ptr[nh] = nc;
}

// order keys: rows with more messages first (key = cap + 1 - min(deg, cap + 1)).
__global__ void k_order_keys(const int32_t* __restrict__ rowptr, int64_t n, int32_t cap,
                             uint32_t* __restrict__ key, int32_t* __restrict__ val) {
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x) {
    int32_t d = rowptr[i + 1] - rowptr[i];
    key[i] = uint32_t(cap + 1 - min(d, cap + 1));
    val[i] = int32_t(i);
  }
}

// slot -> {row, e_begin, e_end, hub_rank} and the row's first 8 sources
// (clamped to the last one): one 16-B + one 32-B load replace the
// order -> hub_rank -> rowptr -> col chain of dependent loads in the tile kernel.
// Also the class boundaries of the tile stage (max over slots of 1 + the slot
// index of every hub / > kLightMax-message slot, of every hub / > 1-message
// slot, of every hub / > kLightLo-message slot, and of every hub /
// > kLightMaxBf16-message slot -- bf16 rows' general / light boundary): exact
// for any slot order.
__global__ void k_slot_desc(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                            int64_t n, const int32_t* __restrict__ order,
                            const int32_t* __restrict__ hub_rank, int4* __restrict__ desc,
                            int32_t* __restrict__ cols8, int64_t* __restrict__ split) {
  unsigned long long s_gen = 0, s_light = 0, s_short = 0, s_gen16 = 0;
  for (int64_t s = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; s < n;
       s += int64_t(gridDim.x) * blockDim.x) {
    const int32_t i = order ? order[s] : int32_t(s);
    const int32_t b = rowptr[i], e = rowptr[i + 1];
    const int32_t hr = hub_rank ? hub_rank[i] : -1;
    desc[s] = make_int4(i, b, e, hr);
    if (cols8) {
#pragma unroll
      for (int k = 0; k < 8; ++k) cols8[s * 8 + k] = col[min(b + k, e - 1)];
    }
    if (hr >= 0 || e - b > kLightMax) s_gen = (unsigned long long)(s + 1);
    if (hr >= 0 || e - b > 1) s_light = (unsigned long long)(s + 1);
    if (hr >= 0 || e - b > kLightLo) s_short = (unsigned long long)(s + 1);
    if (hr >= 0 || e - b > kLightMaxBf16) s_gen16 = (unsigned long long)(s + 1);
  }
  if (split) {
    for (int o = 32; o > 0; o >>= 1) {
      s_gen = max(s_gen, (unsigned long long)__shfl_xor((long long)s_gen, o));
      s_light = max(s_light, (unsigned long long)__shfl_xor((long long)s_light, o));
      s_short = max(s_short, (unsigned long long)__shfl_xor((long long)s_short, o));
      s_gen16 = max(s_gen16, (unsigned long long)__shfl_xor((long long)s_gen16, o));
    }
    if ((threadIdx.x & 63) == 0) {
      if (s_gen) atomicMax(reinterpret_cast<unsigned long long*>(split), s_gen);
      if (s_light) atomicMax(reinterpret_cast<unsigned long long*>(split + 1), s_light);
      if (s_short) atomicMax(reinterpret_cast<unsigned long long*>(split + 2), s_short);
      if (s_gen16) atomicMax(reinterpret_cast<unsigned long long*>(split + 3), s_gen16);
    }
  }
}

// Two independent 64-bit position-sensitive hashes of a COO edge list (sum of
// splitmix64 mixes of (position, src, dst); the sum is order-independent in
// its evaluation, so the block reduction is deterministic in value).
__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

__global__ void k_fingerprint(const int64_t* __restrict__ ei, int64_t E,
                              unsigned long long* __restrict__ out) {
  uint64_t a = 0, b = 0;
  for (int64_t e = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; e < E;
       e += int64_t(gridDim.x) * blockDim.x) {
    const uint64_t s = uint64_t(ei[e]), d = uint64_t(ei[E + e]), p = uint64_t(e);
    a += mix64(p * 0x9E3779B97F4A7C15ull ^ mix64(s + 0x632BE59BD9B4E019ull) ^ (d << 1));
    b += mix64((s * 0xD6E8FEB86659FD93ull + d) ^ mix64(p + 0x85EBCA77C2B2AE63ull));
  }
  for (int o = 32; o > 0; o >>= 1) {
    a += (uint64_t)__shfl_xor((long long)a, o);
    b += (uint64_t)__shfl_xor((long long)b, o);
  }
  if ((threadIdx.x & 63) == 0) {
    atomicAdd(out, (unsigned long long)a);
    atomicAdd(out + 1, (unsigned long long)b);
  }
}

}  // namespace

extern "C" {

gfd_status gfd_coo_fingerprint(const int64_t* edge_index, int64_t num_edges, uint64_t* out,
                               gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (num_edges < 0 || !out || (num_edges > 0 && !edge_index)) return GFD_ERR_ARGUMENT;
  GFD_HIP_CHECK(hipMemsetAsync(out, 0, 2 * sizeof(uint64_t), stream));
  if (num_edges == 0) return GFD_OK;
  k_fingerprint<<<grid_for(num_edges, kBlock, 4096), kBlock, 0, stream>>>(
      edge_index, num_edges, reinterpret_cast<unsigned long long*>(out));
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

gfd_status gfd_plan_desc(const int32_t* rowptr, const int32_t* col, int64_t n,
                         const int32_t* order, const int32_t* hub_rank, int32_t* desc,
                         int32_t* slot_cols, int64_t* class_split, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (n <= 0 || !rowptr || !desc || (slot_cols && !col)) return GFD_ERR_ARGUMENT;
  if (class_split) GFD_HIP_CHECK(hipMemsetAsync(class_split, 0, 4 * sizeof(int64_t), stream));
  k_slot_desc<<<grid_for(n), kBlock, 0, stream>>>(rowptr, col, n, order, hub_rank,
                                                  reinterpret_cast<int4*>(desc), slot_cols,
                                                  class_split);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

const char* gfd_status_string(gfd_status s) {
  switch (s) {
    case GFD_OK: return "ok";
    case GFD_ERR_ARGUMENT: return "invalid argument";
    case GFD_ERR_INDEX: return "edge index out of range [0, num_nodes)";
    case GFD_ERR_WORKSPACE: return "workspace too small";
    case GFD_ERR_HIP: return "HIP runtime error";
    case GFD_ERR_UNSUPPORTED: return "unsupported configuration";
    default: return "unknown status";
  }
}

int gfd_abi_version(void) { return 9; }

static size_t csr_layout(int64_t E, int64_t N, size_t* sort_tmp_out, size_t* scan_tmp_out) {
  size_t sort_tmp = 0, scan_tmp = 0;
  int end_bit = bits_for(N);
  (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t*)nullptr, (uint32_t*)nullptr,
                            (int32_t*)nullptr, (int32_t*)nullptr, size_t(E > 0 ? E : 1), 0, end_bit);
  (void)rocprim::exclusive_scan(nullptr, scan_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                          size_t(N + 1), rocprim::plus<int32_t>());
  if (sort_tmp_out) *sort_tmp_out = sort_tmp;
  if (scan_tmp_out) *scan_tmp_out = scan_tmp;
  Sizer s;
  s.take<uint32_t>(E); s.take<uint32_t>(E); s.take<int32_t>(E); s.take<int32_t>(E);
  s.take<int32_t>(N + 1); s.take<int32_t>(N + 1); s.take<int32_t>(4);
  s.take<char>(sort_tmp); s.take<char>(scan_tmp);
  return s.off;
}

size_t gfd_csr_workspace_size(int64_t num_edges, int64_t num_nodes) {
  if (num_edges < 0 || num_nodes <= 0) return 0;
  return csr_layout(num_edges, num_nodes, nullptr, nullptr);
}

gfd_status gfd_csr_from_coo(const int64_t* edge_index, int64_t E, int64_t N, int32_t* rowptr,
                            int32_t* col, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (N <= 0 || E < 0 || (E > 0 && edge_index == nullptr) || rowptr == nullptr || col == nullptr)
    return GFD_ERR_ARGUMENT;
  if (E + N >= (int64_t(1) << 31) || N >= (int64_t(1) << 31) - 1) return GFD_ERR_UNSUPPORTED;
  size_t sort_tmp, scan_tmp;
  size_t need = csr_layout(E, N, &sort_tmp, &scan_tmp);
  if (ws == nullptr || ws_bytes < need) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  uint32_t* kin = c.take<uint32_t>(E);
  uint32_t* kout = c.take<uint32_t>(E);
  int32_t* vin = c.take<int32_t>(E);
  int32_t* vout = c.take<int32_t>(E);
  int32_t* deg = c.take<int32_t>(N + 1);
  int32_t* cnt = c.take<int32_t>(N + 1);
  int32_t* err = c.take<int32_t>(4);
  void* sort_buf = c.take<char>(sort_tmp);
  void* scan_buf = c.take<char>(scan_tmp);
  if (!c.ok) return GFD_ERR_WORKSPACE;

  GFD_HIP_CHECK(hipMemsetAsync(deg, 0, sizeof(int32_t) * (N + 1), stream));
  GFD_HIP_CHECK(hipMemsetAsync(err, 0, sizeof(int32_t) * 4, stream));
  if (E > 0) {
    k_coo_keys<<<grid_for(E), kBlock, 0, stream>>>(edge_index, E, N, kin, vin, deg, err);
    GFD_LAUNCH_CHECK();
    size_t st = sort_tmp;
    if (rocprim::radix_sort_pairs(sort_buf, st, kin, kout, vin, vout, size_t(E), 0, bits_for(N),
                                  stream) != hipSuccess)
      return GFD_ERR_HIP;
  }
  k_plus_one<<<grid_for(N + 1), kBlock, 0, stream>>>(deg, cnt, N);
  GFD_LAUNCH_CHECK();
  size_t sc = scan_tmp;
  if (rocprim::exclusive_scan(scan_buf, sc, cnt, rowptr, 0, size_t(N + 1), rocprim::plus<int32_t>(),
                              stream) != hipSuccess)
    return GFD_ERR_HIP;
  k_fill_col<<<grid_for(E > N ? E : N), kBlock, 0, stream>>>(kout, vout, E, N, rowptr, col);
  GFD_LAUNCH_CHECK();
  int32_t herr = 0;
  GFD_HIP_CHECK(hipMemcpyAsync(&herr, err, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
  GFD_HIP_CHECK(hipStreamSynchronize(stream));
  return herr ? GFD_ERR_INDEX : GFD_OK;
}

static size_t csc_layout(int64_t M, int64_t N, size_t* sort_tmp_out, size_t* scan_tmp_out) {
  size_t sort_tmp = 0, scan_tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t*)nullptr, (uint32_t*)nullptr,
                            (int32_t*)nullptr, (int32_t*)nullptr, size_t(M > 0 ? M : 1), 0,
                            bits_for(N));
  (void)rocprim::exclusive_scan(nullptr, scan_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                          size_t(N + 1), rocprim::plus<int32_t>());
  if (sort_tmp_out) *sort_tmp_out = sort_tmp;
  if (scan_tmp_out) *scan_tmp_out = scan_tmp;
  Sizer s;
  s.take<uint32_t>(M); s.take<uint32_t>(M); s.take<int32_t>(M); s.take<int32_t>(M);
  s.take<int32_t>(N + 1); s.take<char>(sort_tmp); s.take<char>(scan_tmp);
  return s.off;
}

size_t gfd_csc_workspace_size(int64_t num_messages, int64_t num_nodes) {
  if (num_messages < 0 || num_nodes <= 0) return 0;
  return csc_layout(num_messages, num_nodes, nullptr, nullptr);
}

gfd_status gfd_csc_from_csr(const int32_t* rowptr, const int32_t* col, int64_t M, int64_t N,
                            int32_t* colptr, int32_t* csc_dst, int32_t* csc_eid, void* ws,
                            size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (N <= 0 || M <= 0 || !rowptr || !col || !colptr || !csc_dst || !csc_eid) return GFD_ERR_ARGUMENT;
  size_t sort_tmp, scan_tmp;
  size_t need = csc_layout(M, N, &sort_tmp, &scan_tmp);
  if (ws == nullptr || ws_bytes < need) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  uint32_t* kin = c.take<uint32_t>(M);
  uint32_t* kout = c.take<uint32_t>(M);
  int32_t* vin = c.take<int32_t>(M);
  int32_t* rowid = c.take<int32_t>(M);
  int32_t* cnt = c.take<int32_t>(N + 1);
  void* sort_buf = c.take<char>(sort_tmp);
  void* scan_buf = c.take<char>(scan_tmp);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  GFD_HIP_CHECK(hipMemsetAsync(cnt, 0, sizeof(int32_t) * (N + 1), stream));
  k_csr_keys<<<grid_for(M), kBlock, 0, stream>>>(col, M, kin, vin, cnt);
  GFD_LAUNCH_CHECK();
  size_t st = sort_tmp;
  if (rocprim::radix_sort_pairs(sort_buf, st, kin, kout, vin, csc_eid, size_t(M), 0, bits_for(N),
                                stream) != hipSuccess)
    return GFD_ERR_HIP;
  size_t sc = scan_tmp;
  if (rocprim::exclusive_scan(scan_buf, sc, cnt, colptr, 0, size_t(N + 1), rocprim::plus<int32_t>(),
                              stream) != hipSuccess)
    return GFD_ERR_HIP;
  k_row_of<<<grid_for(N * 64), kBlock, 0, stream>>>(rowptr, N, rowid);
  GFD_LAUNCH_CHECK();
  k_gather_dst<<<grid_for(M), kBlock, 0, stream>>>(csc_eid, rowid, M, csc_dst);
  GFD_LAUNCH_CHECK();
  return GFD_OK;
}

static size_t plan_layout(int64_t n, size_t* scan_tmp_out) {
  size_t scan_tmp = 0;
  (void)rocprim::exclusive_scan(nullptr, scan_tmp, (const int32_t*)nullptr, (int32_t*)nullptr, 0,
                          size_t(n + 1), rocprim::plus<int32_t>());
  if (scan_tmp_out) *scan_tmp_out = scan_tmp;
  Sizer s;
  s.take<int32_t>(n + 1); s.take<int32_t>(n + 1); s.take<int32_t>(n + 1); s.take<int32_t>(n + 1);
  s.take<int64_t>(2); s.take<char>(scan_tmp); s.take<char>(scan_tmp);
  return s.off;
}

size_t gfd_plan_workspace_size(int64_t num_dst) {
  if (num_dst <= 0) return 0;
  return plan_layout(num_dst, nullptr);
}

gfd_status gfd_plan_hubs(const int32_t* rowptr, int64_t n, int32_t thr, int32_t chunk,
                         int32_t* hub_rank, int32_t* hub_chunk, int32_t* hub_chunk_ptr,
                         int32_t* hub_dst, int64_t max_hubs, int64_t max_chunks, int64_t* num_hubs,
                         int64_t* num_chunks, void* ws, size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (n <= 0 || !rowptr || !hub_rank || !num_hubs || !num_chunks || thr < 1 || chunk < 1)
    return GFD_ERR_ARGUMENT;
  if ((max_hubs > 0 && (!hub_dst || !hub_chunk_ptr)) || (max_chunks > 0 && !hub_chunk))
    return GFD_ERR_ARGUMENT;
  size_t scan_tmp;
  size_t need = plan_layout(n, &scan_tmp);
  if (ws == nullptr || ws_bytes < need) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  int32_t* is_hub = c.take<int32_t>(n + 1);
  int32_t* nchunk = c.take<int32_t>(n + 1);
  int32_t* hub_idx = c.take<int32_t>(n + 1);
  int32_t* chunk_off = c.take<int32_t>(n + 1);
  int64_t* counts = c.take<int64_t>(2);
  void* scan_a = c.take<char>(scan_tmp);
  void* scan_b = c.take<char>(scan_tmp);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  k_hub_flags<<<grid_for(n + 1), kBlock, 0, stream>>>(rowptr, n, thr, chunk, is_hub, nchunk);
  GFD_LAUNCH_CHECK();
  size_t sa = scan_tmp, sb = scan_tmp;
  if (rocprim::exclusive_scan(scan_a, sa, is_hub, hub_idx, 0, size_t(n + 1), rocprim::plus<int32_t>(),
                              stream) != hipSuccess)
    return GFD_ERR_HIP;
  if (rocprim::exclusive_scan(scan_b, sb, nchunk, chunk_off, 0, size_t(n + 1),
                              rocprim::plus<int32_t>(), stream) != hipSuccess)
    return GFD_ERR_HIP;
  k_hub_write<<<grid_for(n), kBlock, 0, stream>>>(rowptr, n, thr, chunk, hub_idx, chunk_off, hub_rank,
                                                 hub_chunk, hub_chunk_ptr, hub_dst, max_hubs,
                                                 max_chunks);
  GFD_LAUNCH_CHECK();
  k_hub_tail<<<1, 1, 0, stream>>>(hub_idx, chunk_off, n, max_hubs > 0 ? hub_chunk_ptr : nullptr,
                                  max_hubs, counts);
  GFD_LAUNCH_CHECK();
  int64_t h[2];
  GFD_HIP_CHECK(hipMemcpyAsync(h, counts, sizeof(h), hipMemcpyDeviceToHost, stream));
  GFD_HIP_CHECK(hipStreamSynchronize(stream));
  *num_hubs = h[0];
  *num_chunks = h[1];
  if (h[0] > max_hubs || h[1] > max_chunks) return GFD_ERR_WORKSPACE;
  return GFD_OK;
}

static size_t order_layout(int64_t n, int32_t cap, size_t* sort_tmp_out) {
  size_t sort_tmp = 0;
  (void)rocprim::radix_sort_pairs(nullptr, sort_tmp, (uint32_t*)nullptr, (uint32_t*)nullptr,
                                  (int32_t*)nullptr, (int32_t*)nullptr, size_t(n > 0 ? n : 1), 0,
                                  bits_for(int64_t(cap) + 1));
  if (sort_tmp_out) *sort_tmp_out = sort_tmp;
  Sizer s;
  s.take<uint32_t>(n); s.take<uint32_t>(n); s.take<int32_t>(n); s.take<char>(sort_tmp);
  return s.off;
}

size_t gfd_order_workspace_size(int64_t num_dst, int32_t cap) {
  if (num_dst <= 0 || cap < 1) return 0;
  return order_layout(num_dst, cap, nullptr);
}

gfd_status gfd_plan_order(const int32_t* rowptr, int64_t n, int32_t cap, int32_t* order, void* ws,
                          size_t ws_bytes, gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (n <= 0 || cap < 1 || !rowptr || !order) return GFD_ERR_ARGUMENT;
  size_t sort_tmp;
  size_t need = order_layout(n, cap, &sort_tmp);
  if (ws == nullptr || ws_bytes < need) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  uint32_t* kin = c.take<uint32_t>(n);
  uint32_t* kout = c.take<uint32_t>(n);
  int32_t* vin = c.take<int32_t>(n);
  void* sort_buf = c.take<char>(sort_tmp);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  k_order_keys<<<grid_for(n), kBlock, 0, stream>>>(rowptr, n, cap, kin, vin);
  GFD_LAUNCH_CHECK();
  size_t st = sort_tmp;
  if (rocprim::radix_sort_pairs(sort_buf, st, kin, kout, vin, order, size_t(n), 0,
                                bits_for(int64_t(cap) + 1), stream) != hipSuccess)
    return GFD_ERR_HIP;
  return GFD_OK;
}

}  // extern "C"
