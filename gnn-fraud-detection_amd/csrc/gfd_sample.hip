// gfd_sample.hip -- GPU neighbour sampling for the reference's mini-batch mode
// (SURVEY.md §8f rank 3): PyG NeighborLoader(data, num_neighbors=[10, 10, 10],
// batch_size=256, input_nodes=mask, shuffle=...) at
// /root/reference/src/data/dataloader.py:42-66 (config.py:41).
//
// Per batch: the seeds are the first nodes of the sampled subgraph; hop l
// samples, for every node of frontier l, up to k_l of its in-neighbours (the
// sources j of edges j -> i; message flow source -> target) uniformly WITHOUT
// replacement (all of them when the in-degree is <= k_l), PyG's default
// (replace=False, directed).  Sources not yet in the subgraph are appended in
// order of first appearance and form frontier l + 1.  Output: n_id (global ids
// of the subgraph's nodes), the sampled edges with local ids.
//
// Sampling is Robert Floyd's algorithm: k draws, O(k^2) work per node whatever
// its degree (a 100k-message hub costs the same as a 20-message node), with
// counter-based random numbers (splitmix64 of seed, hop, node, draw), so one
// thread per frontier node and the result is a deterministic function of the
// seed -- the CPU restatement (oracle/sample_ref.py) reproduces it bit for bit.
// PyG's own random stream cannot be reproduced (different generator), so the
// distribution, not the draw, is what matches PyG (tests: uniformity).
//
// First appearance is made deterministic without ordering the atomics: every
// candidate has a position p in (frontier order, draw order); a node's first
// position is the atomicMin over its candidates; a prefix sum over "p is the
// first position of a node not yet in the subgraph" numbers the new nodes.
// local_of[N] (the global -> local map) is all -1 between batches: the call
// clears exactly the entries it set.
#include <rocprim/device/device_scan.hpp>

#include "gfd_common.h"

using namespace gfd;

namespace {

constexpr int kSB = 256;
constexpr int kMaxFanout = 64;

inline int sgrid(int64_t n) {
  int64_t g = (n + kSB - 1) / kSB;
  return int(g < 1 ? 1 : (g < 65536 ? g : 65536));
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// uniform draw in [0, m] for (seed, hop, node, draw)
__device__ __forceinline__ int64_t draw(uint64_t seed, int hop, int64_t node, int i, int64_t m) {
  const uint64_t z = mix64(seed ^ (uint64_t(hop + 1) * 0x9E3779B97F4A7C15ull) ^
                           (uint64_t(node) * 0xD1B54A32D192ED03ull) ^
                           (uint64_t(i + 1) * 0x8CB92BA72F3D8DD7ull));
  return int64_t(z % uint64_t(m + 1));
}

// in-degree of node i in the sampling CSR (the GATConv CSR minus the self loop
// appended last in every segment)
__device__ __forceinline__ int64_t in_deg(const int32_t* rowptr, int64_t i) {
  return int64_t(rowptr[i + 1]) - rowptr[i] - 1;
}

// frontier f_lo .. f_hi (device counts): cnt[f] = min(k, in-degree)
__global__ void k_counts(const int32_t* __restrict__ rowptr, const int64_t* __restrict__ n_id,
                         const int64_t* __restrict__ lvl, int hop, int k, int64_t max_f,
                         int64_t* __restrict__ cnt) {
  const int64_t f0 = lvl[hop], f1 = lvl[hop + 1];
  for (int64_t f = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; f < max_f;
       f += int64_t(gridDim.x) * blockDim.x) {
    int64_t c = 0;
    if (f0 + f < f1) {
      const int64_t d = in_deg(rowptr, n_id[f0 + f]);
      c = d < k ? d : k;
    }
    cnt[f] = c;
  }
}

// Floyd sampling: candidates at off[f] .. off[f] + cnt[f]
__global__ void k_floyd(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ col,
                        const int64_t* __restrict__ n_id, const int64_t* __restrict__ lvl, int hop,
                        int k, uint64_t seed, int64_t max_f, const int64_t* __restrict__ off,
                        int64_t* __restrict__ cand, int64_t* __restrict__ cand_dst,
                        int64_t* __restrict__ cand_eid) {
  const int64_t f0 = lvl[hop], f1 = lvl[hop + 1];
  for (int64_t f = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; f < max_f && f0 + f < f1;
       f += int64_t(gridDim.x) * blockDim.x) {
    const int64_t node = n_id[f0 + f];
    const int64_t e0 = rowptr[node];
    const int64_t d = in_deg(rowptr, node);
    const int64_t o = off[f];
    if (d <= k) {  // every in-neighbour
      for (int64_t t = 0; t < d; ++t) {
        cand[o + t] = col[e0 + t];
        cand_dst[o + t] = f0 + f;
        cand_eid[o + t] = e0 + t;
      }
      continue;
    }
    int64_t pick[kMaxFanout];
    for (int i = 0; i < k; ++i) {
      const int64_t j = d - k + i;
      int64_t t = draw(seed, hop, node, i, j);
      for (int q = 0; q < i; ++q)
        if (pick[q] == t) { t = j; break; }
      pick[i] = t;
      cand[o + i] = col[e0 + t];
      cand_dst[o + i] = f0 + f;
      cand_eid[o + i] = e0 + t;
    }
  }
}

__global__ void k_first(const int64_t* __restrict__ cand, const int64_t* __restrict__ ncand,
                        int64_t max_c, const int32_t* __restrict__ local_of,
                        int64_t* __restrict__ first) {
  const int64_t n = *ncand;
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < max_c && p < n;
       p += int64_t(gridDim.x) * blockDim.x) {
    const int64_t j = cand[p];
    if (local_of[j] < 0) atomicMin(reinterpret_cast<unsigned long long*>(first + j),
                                   static_cast<unsigned long long>(p));
  }
}

__global__ void k_flags(const int64_t* __restrict__ cand, const int64_t* __restrict__ ncand,
                        int64_t max_c, const int32_t* __restrict__ local_of,
                        const int64_t* __restrict__ first, int64_t* __restrict__ flag) {
  const int64_t n = *ncand;
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < max_c;
       p += int64_t(gridDim.x) * blockDim.x) {
    int64_t v = 0;
    if (p < n) {
      const int64_t j = cand[p];
      v = (local_of[j] < 0 && first[j] == p) ? 1 : 0;
    }
    flag[p] = v;
  }
}

// new nodes get local ids lvl[hop + 1] + rank; the next level ends after them
__global__ void k_assign(const int64_t* __restrict__ cand, const int64_t* __restrict__ ncand,
                         int64_t max_c, const int64_t* __restrict__ flag,
                         const int64_t* __restrict__ rank, int64_t* __restrict__ lvl, int hop,
                         int64_t* __restrict__ n_id, int32_t* __restrict__ local_of,
                         int64_t* __restrict__ first) {
  const int64_t n = *ncand;
  const int64_t base = lvl[hop + 1];
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < max_c && p < n;
       p += int64_t(gridDim.x) * blockDim.x) {
    if (flag[p]) {
      const int64_t j = cand[p];
      const int64_t li = base + rank[p];
      n_id[li] = j;
      local_of[j] = int32_t(li);
      first[j] = INT64_MAX;
    }
  }
}

__global__ void k_level_end(const int64_t* __restrict__ ncand, int64_t max_c,
                            const int64_t* __restrict__ flag, const int64_t* __restrict__ rank,
                            int64_t* __restrict__ lvl, int hop) {
  const int64_t n = *ncand;
  lvl[hop + 2] = lvl[hop + 1] + (n > 0 ? rank[n - 1] + flag[n - 1] : 0);
  (void)max_c;
}

__global__ void k_edges(const int64_t* __restrict__ cand, const int64_t* __restrict__ cand_dst,
                        const int64_t* __restrict__ cand_eid, const int64_t* __restrict__ ncand,
                        int64_t max_c, const int32_t* __restrict__ local_of,
                        const int64_t* __restrict__ edge_ptr, int hop, int64_t* __restrict__ esrc,
                        int64_t* __restrict__ edst, int64_t* __restrict__ eid) {
  const int64_t n = *ncand;
  const int64_t base = edge_ptr[hop];
  for (int64_t p = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; p < max_c && p < n;
       p += int64_t(gridDim.x) * blockDim.x) {
    esrc[base + p] = local_of[cand[p]];
    edst[base + p] = cand_dst[p];
    eid[base + p] = cand_eid[p];
  }
}

__global__ void k_total(const int64_t* __restrict__ cnt, const int64_t* __restrict__ off,
                        int64_t m, int64_t* __restrict__ ncand) {
  *ncand = off[m - 1] + cnt[m - 1];
}

__global__ void k_edge_ptr(const int64_t* __restrict__ ncand, int64_t* __restrict__ edge_ptr,
                           int hop) {
  edge_ptr[hop + 1] = edge_ptr[hop] + *ncand;
}

__global__ void k_seed(const int64_t* __restrict__ seeds, int64_t ns, int64_t N,
                       int64_t* __restrict__ n_id, int32_t* __restrict__ local_of,
                       int32_t* __restrict__ err) {
  for (int64_t s = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; s < ns;
       s += int64_t(gridDim.x) * blockDim.x) {
    const int64_t j = seeds[s];
    if (j < 0 || j >= N) { atomicOr(err, 1); n_id[s] = 0; continue; }
    n_id[s] = j;
    local_of[j] = int32_t(s);  // seeds are distinct (NeighborLoader input nodes)
  }
}

__global__ void k_init(int64_t* __restrict__ level_ptr, int64_t* __restrict__ edge_ptr,
                       int64_t ns) {
  level_ptr[0] = 0;
  level_ptr[1] = ns;
  edge_ptr[0] = 0;
}

__global__ void k_clear(const int64_t* __restrict__ n_id, const int64_t* __restrict__ lvl,
                        int hops, int32_t* __restrict__ local_of) {
  const int64_t n = lvl[hops + 1];
  for (int64_t i = blockIdx.x * int64_t(blockDim.x) + threadIdx.x; i < n;
       i += int64_t(gridDim.x) * blockDim.x)
    local_of[n_id[i]] = -1;
}

size_t scan_tmp(int64_t n) {
  size_t t = 0;
  (void)rocprim::exclusive_scan(nullptr, t, (const int64_t*)nullptr, (int64_t*)nullptr,
                                int64_t(0), size_t(n > 0 ? n : 1), rocprim::plus<int64_t>());
  return t;
}

// worst-case sizes: frontier l <= seeds * prod(k_0..k_{l-1}), capped by N
void bounds(int64_t ns, const int32_t* fan, int hops, int64_t N, int64_t* max_f, int64_t* max_c,
            int64_t* max_nodes, int64_t* max_edges) {
  int64_t f = ns, nodes = ns, edges = 0, mf = ns, mc = 1;
  for (int l = 0; l < hops; ++l) {
    const int64_t c = f * fan[l];
    mc = c > mc ? c : mc;
    edges += c;
    f = c < N ? c : N;
    mf = f > mf ? f : mf;
    nodes += f;
  }
  *max_f = mf;
  *max_c = mc;
  *max_nodes = nodes < N ? nodes : N;
  *max_edges = edges;
}

size_t sample_layout(int64_t N, int64_t max_f, int64_t max_c, size_t* st) {
  *st = scan_tmp(max_c > max_f ? max_c : max_f);
  Sizer s;
  s.take<int64_t>(max_f);       // counts
  s.take<int64_t>(max_f + 1);   // offsets
  s.take<int64_t>(max_c);       // cand
  s.take<int64_t>(max_c);       // cand_dst
  s.take<int64_t>(max_c);       // cand_eid
  s.take<int64_t>(max_c);       // flag
  s.take<int64_t>(max_c);       // rank
  s.take<int64_t>(N);           // first
  s.take<int64_t>(4);           // ncand
  s.take<int32_t>(4);           // err
  s.take<char>(*st);
  return s.off;
}

}  // namespace

extern "C" {

size_t gfd_sample_workspace_size(int64_t num_nodes, int64_t num_seeds, const int32_t* fanouts,
                                 int32_t num_hops) {
  if (num_nodes <= 0 || num_seeds <= 0 || num_hops <= 0 || !fanouts) return 0;
  int64_t mf, mc, mn, me;
  bounds(num_seeds, fanouts, num_hops, num_nodes, &mf, &mc, &mn, &me);
  size_t st;
  return sample_layout(num_nodes, mf, mc, &st);
}

gfd_status gfd_sample_bounds(int64_t num_nodes, int64_t num_seeds, const int32_t* fanouts,
                             int32_t num_hops, int64_t* max_nodes, int64_t* max_edges) {
  if (num_nodes <= 0 || num_seeds <= 0 || num_hops <= 0 || !fanouts || !max_nodes || !max_edges)
    return GFD_ERR_ARGUMENT;
  for (int l = 0; l < num_hops; ++l)
    if (fanouts[l] < 0 || fanouts[l] > kMaxFanout) return GFD_ERR_UNSUPPORTED;
  int64_t mf, mc;
  bounds(num_seeds, fanouts, num_hops, num_nodes, &mf, &mc, max_nodes, max_edges);
  return GFD_OK;
}

gfd_status gfd_sample_neighbors(const int32_t* rowptr, const int32_t* col, int64_t N,
                                const int64_t* seeds, int64_t ns, const int32_t* fanouts,
                                int32_t hops, uint64_t seed, int32_t* local_of, int64_t* n_id,
                                int64_t* level_ptr, int64_t* edge_src, int64_t* edge_dst,
                                int64_t* edge_id, int64_t* edge_ptr, void* ws, size_t ws_bytes,
                                gfd_stream_t stream_) {
  hipStream_t stream = static_cast<hipStream_t>(stream_);
  if (!rowptr || !col || N <= 0 || !seeds || ns <= 0 || !fanouts || hops <= 0 || !local_of ||
      !n_id || !level_ptr || !edge_src || !edge_dst || !edge_id || !edge_ptr)
    return GFD_ERR_ARGUMENT;
  for (int l = 0; l < hops; ++l)
    if (fanouts[l] < 0 || fanouts[l] > kMaxFanout) return GFD_ERR_UNSUPPORTED;
  int64_t mf, mc, mn, me;
  bounds(ns, fanouts, hops, N, &mf, &mc, &mn, &me);
  size_t st;
  if (!ws || ws_bytes < sample_layout(N, mf, mc, &st)) return GFD_ERR_WORKSPACE;
  Carve c(ws, ws_bytes);
  int64_t* cnt = c.take<int64_t>(mf);
  int64_t* off = c.take<int64_t>(mf + 1);
  int64_t* cand = c.take<int64_t>(mc);
  int64_t* cand_dst = c.take<int64_t>(mc);
  int64_t* cand_eid = c.take<int64_t>(mc);
  int64_t* flag = c.take<int64_t>(mc);
  int64_t* rank = c.take<int64_t>(mc);
  int64_t* first = c.take<int64_t>(N);
  int64_t* ncand = c.take<int64_t>(4);
  int32_t* err = c.take<int32_t>(4);
  void* tmp = c.take<char>(st);
  if (!c.ok) return GFD_ERR_WORKSPACE;
  GFD_HIP_CHECK(hipMemsetAsync(err, 0, sizeof(int32_t) * 4, stream));
  GFD_HIP_CHECK(hipMemsetAsync(first, 0x7f, sizeof(int64_t) * N, stream));  // > any position
  // seeds: level 0 = [0, ns); no edges yet
  k_init<<<1, 1, 0, stream>>>(level_ptr, edge_ptr, ns);
  GFD_LAUNCH_CHECK();
  k_seed<<<sgrid(ns), kSB, 0, stream>>>(seeds, ns, N, n_id, local_of, err);
  GFD_LAUNCH_CHECK();
  for (int l = 0; l < hops; ++l) {
    const int k = fanouts[l];
    k_counts<<<sgrid(mf), kSB, 0, stream>>>(rowptr, n_id, level_ptr, l, k, mf, cnt);
    GFD_LAUNCH_CHECK();
    size_t t = st;
    if (rocprim::exclusive_scan(tmp, t, cnt, off, int64_t(0), size_t(mf),
                                rocprim::plus<int64_t>(), stream) != hipSuccess)
      return GFD_ERR_HIP;
    k_total<<<1, 1, 0, stream>>>(cnt, off, mf, ncand);
    GFD_LAUNCH_CHECK();
    k_floyd<<<sgrid(mf), kSB, 0, stream>>>(rowptr, col, n_id, level_ptr, l, k, seed, mf, off,
                                           cand, cand_dst, cand_eid);
    GFD_LAUNCH_CHECK();
    k_first<<<sgrid(mc), kSB, 0, stream>>>(cand, ncand, mc, local_of, first);
    GFD_LAUNCH_CHECK();
    k_flags<<<sgrid(mc), kSB, 0, stream>>>(cand, ncand, mc, local_of, first, flag);
    GFD_LAUNCH_CHECK();
    t = st;
    if (rocprim::exclusive_scan(tmp, t, flag, rank, int64_t(0), size_t(mc),
                                rocprim::plus<int64_t>(), stream) != hipSuccess)
      return GFD_ERR_HIP;
    k_assign<<<sgrid(mc), kSB, 0, stream>>>(cand, ncand, mc, flag, rank, level_ptr, l, n_id,
                                            local_of, first);
    GFD_LAUNCH_CHECK();
    k_level_end<<<1, 1, 0, stream>>>(ncand, mc, flag, rank, level_ptr, l);
    GFD_LAUNCH_CHECK();
    k_edges<<<sgrid(mc), kSB, 0, stream>>>(cand, cand_dst, cand_eid, ncand, mc, local_of,
                                           edge_ptr, l, edge_src, edge_dst, edge_id);
    GFD_LAUNCH_CHECK();
    k_edge_ptr<<<1, 1, 0, stream>>>(ncand, edge_ptr, l);
    GFD_LAUNCH_CHECK();
  }
  // leave local_of all -1 for the next batch
  k_clear<<<sgrid(mn), kSB, 0, stream>>>(n_id, level_ptr, hops, local_of);
  GFD_LAUNCH_CHECK();
  int32_t herr = 0;
  GFD_HIP_CHECK(hipMemcpyAsync(&herr, err, sizeof(int32_t), hipMemcpyDeviceToHost, stream));
  GFD_HIP_CHECK(hipStreamSynchronize(stream));
  return herr ? GFD_ERR_INDEX : GFD_OK;
}

}  // extern "C"
