/*
 * gfd.h -- C ABI of the MI355X-native GATConv engine (libgfd.so, gfx950).
 *
 * This is the drop-in boundary for the reference's hot path: the
 * ``torch_geometric.nn.GATConv`` operator that the reference imports at
 * /root/reference/src/models/gat.py:4 and tgn.py:4, constructs as
 * ``GATConv(in, 64, heads=8, concat=False, dropout=p)`` (gat.py:39,45,51;
 * tgn.py:43,49,55) and calls as ``gat(h, edge_index)`` (gat.py:80, tgn.py:94).
 * PyG's GATConv is third-party (setup.py:13, unpinned); the interface each entry
 * point replaces is named next to it.  Plain pointers and sizes only: no torch
 * types, no HIP headers (a stream is passed as an opaque ``hipStream_t``
 * handle), so ctypes / cgo / JNI bind it as-is.
 *
 * Conventions
 *  - Every pointer except the ``ws`` workspace and explicitly host-side
 *    arguments is a DEVICE pointer on the current HIP device.
 *  - The caller owns all memory, including workspaces; the library allocates
 *    nothing and keeps no global state.  All work is enqueued on ``stream``;
 *    nothing synchronises except where a function says so.
 *  - Node features x are fp32 (GFD_DTYPE_F32, configs C1-C4) or bf16
 *    (GFD_DTYPE_BF16, config C5), row-major with any row pitch; every other
 *    floating-point argument is IEEE fp32.  Internally the feature projection
 *    runs on f16 MFMA with a 3-term hi/lo split over power-of-two scaled rows
 *    (~2^-21 relative, fp32-faithful); the logits s = x.U, t = x.V (U, V the
 *    folded att . W vectors) use the same 3-term f16 split on MFMA; softmax,
 *    aggregation and accumulation are fp32.  A bf16 x is converted exactly on
 *    load, so the result is the fp32 forward of the bf16-rounded features.
 *  - Graph layout: ``edge_index`` is the reference's COO ``int64 [2, E]``
 *    (dataset.py:104; row 0 = source j, row 1 = destination i, flow
 *    source->target).  Internally a destination-sorted CSR of int32 with the
 *    PyG self-loop policy (existing self loops removed, one appended per node,
 *    duplicates kept): ``rowptr[N+1]``, ``col[E']``, E' = E - loops + N.
 */
#ifndef GFD_H
#define GFD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* gfd_stream_t; /* a hipStream_t; NULL = the null stream */
typedef int32_t gfd_status;

#define GFD_OK 0
#define GFD_ERR_ARGUMENT 1    /* null pointer, bad shape, size out of range  (PyG/ATen: ValueError)   */
#define GFD_ERR_INDEX 2       /* an edge index outside [0, N)                (ATen: index out of range) */
#define GFD_ERR_WORKSPACE 3   /* ws_bytes smaller than the *_workspace_size answer                     */
#define GFD_ERR_HIP 4         /* a HIP runtime call or kernel launch failed                            */
#define GFD_ERR_UNSUPPORTED 5 /* heads/channels/features outside the compiled set (H=8, C=64, F<=256)  */

/* Element type of the node features x (``x_dtype`` arguments). */
#define GFD_DTYPE_F32 0
#define GFD_DTYPE_BF16 1

const char* gfd_status_string(gfd_status status);
int gfd_abi_version(void);
/* Provenance: "gfd-src-sha256:<SHA-256 of the library's sources, headers,
 * flags> <target>" (gnn-fraud-detection_amd/gfd/build.py source_id). */
const char* gfd_build_id(void);

/* ---------------------------------------------------------------------------
 * Graph formats.  Replaces PyG's per-call remove_self_loops + add_self_loops
 * (inside GATConv.forward) and the COO gather/scatter index math.
 * ------------------------------------------------------------------------- */

/* Workspace for gfd_csr_from_coo (device bytes). */
size_t gfd_csr_workspace_size(int64_t num_edges, int64_t num_nodes);

/* COO [2,E] int64 -> destination-sorted CSR.  ``col`` must hold E + N entries;
 * on return rowptr[N] = E'.  Within a destination the original edge order is
 * kept (stable), and the self loop is last -- PyG's message order.
 * Validates every index; synchronises ``stream`` once to report
 * GFD_ERR_INDEX.  Not for the timed path: build once per graph and cache. */
gfd_status gfd_csr_from_coo(const int64_t* edge_index, int64_t num_edges, int64_t num_nodes,
                            int32_t* rowptr, int32_t* col, void* ws, size_t ws_bytes,
                            gfd_stream_t stream);

/* Graph ingest (replaces the id -> index dict and the per-row loops of
 * EllipticBitcoinDataset.process, dataset.py:75-129).  gfd_id_map_build sorts
 * (id, position) pairs of the node id column (stable: a repeated id maps to
 * its LAST position, like the reference's dict comprehension, :92);
 * gfd_id_map_lookup maps query ids to positions (-1 when unknown);
 * gfd_edges_from_ids keeps the edges whose two endpoint ids are known, in
 * their original order (:95-101), as int64 COO edge_index [2, E] (row stride
 * E; the first *num_kept columns are written; num_kept is a device int64). */
size_t gfd_id_map_workspace_size(int64_t num_ids);
gfd_status gfd_id_map_build(const int64_t* ids, int64_t num_ids, int64_t* sorted_ids,
                            int32_t* sorted_idx, void* ws, size_t ws_bytes, gfd_stream_t stream);
gfd_status gfd_id_map_lookup(const int64_t* sorted_ids, const int32_t* sorted_idx, int64_t num_ids,
                             const int64_t* queries, int64_t num_queries, int32_t* out,
                             gfd_stream_t stream);
size_t gfd_edges_from_ids_workspace_size(int64_t num_edges);
gfd_status gfd_edges_from_ids(const int64_t* sorted_ids, const int32_t* sorted_idx,
                              int64_t num_ids, const int64_t* src_ids, const int64_t* dst_ids,
                              int64_t num_edges, int64_t* edge_index, int64_t* num_kept, void* ws,
                              size_t ws_bytes, gfd_stream_t stream);

/* 128-bit fingerprint of a COO edge list (two independent position-sensitive
 * 64-bit hashes of every (position, src, dst), device out[2]; no sync).  The
 * graph cache keys on it so that a re-uploaded but equal edge_index (the
 * reference's per-epoch batch.to(device), train.py:105) reuses its CSR. */
gfd_status gfd_coo_fingerprint(const int64_t* edge_index, int64_t num_edges, uint64_t* out,
                               gfd_stream_t stream);

/* Source-sorted view of a CSR (for the backward scatter to sources):
 * colptr[N+1]; for the k-th message leaving source j (stable in CSR order),
 * csc_dst[colptr[j]+k] = its destination and csc_eid[...] = its CSR position. */
size_t gfd_csc_workspace_size(int64_t num_messages, int64_t num_nodes);
gfd_status gfd_csc_from_csr(const int32_t* rowptr, const int32_t* col, int64_t num_messages,
                            int64_t num_nodes, int32_t* colptr, int32_t* csc_dst, int32_t* csc_eid,
                            void* ws, size_t ws_bytes, gfd_stream_t stream);

/* Hub plan: destinations with more than ``hub_threshold`` messages are split
 * into chunks of at most ``chunk`` messages processed by separate waves and
 * merged.  Writes (device) hub_rank[num_dst] (-1 light, else hub index),
 * hub_chunk[4*max_chunks] ({hub, e_begin, e_end, dst}), hub_chunk_ptr[n_hubs+1],
 * hub_dst[n_hubs], and the HOST counters *num_hubs, *num_chunks.  Synchronises
 * the stream once.  ``max_chunks``/``max_hubs`` bound the arrays; if exceeded
 * it returns GFD_ERR_WORKSPACE with the needed counts in the host counters. */
size_t gfd_plan_workspace_size(int64_t num_dst);
gfd_status gfd_plan_hubs(const int32_t* rowptr, int64_t num_dst, int32_t hub_threshold,
                         int32_t chunk, int32_t* hub_rank, int32_t* hub_chunk,
                         int32_t* hub_chunk_ptr, int32_t* hub_dst, int64_t max_hubs,
                         int64_t max_chunks, int64_t* num_hubs, int64_t* num_chunks, void* ws,
                         size_t ws_bytes, gfd_stream_t stream);

/* Tile order: destination ids sorted by descending message count (capped at
 * cap + 1, stable), so each 16-destination tile of the fused kernel holds rows
 * of similar length (no tile waits on one long row).  order[num_dst]. */
size_t gfd_order_workspace_size(int64_t num_dst, int32_t cap);
gfd_status gfd_plan_order(const int32_t* rowptr, int64_t num_dst, int32_t cap, int32_t* order,
                          void* ws, size_t ws_bytes, gfd_stream_t stream);

/* Slot descriptors: desc[4*s .. 4*s+3] = {row, e_begin, e_end, hub_rank} of
 * tile slot s (row = order[s], or s when order is NULL; hub_rank -1 when
 * NULL) and, when slot_cols is not NULL, slot_cols[8*s + k] = col[min(e_begin
 * + k, e_end - 1)] (the first 8 sources, prefetched one tile ahead).
 * class_split (nullable, device int64[4]; ABI 9 -- [3] in ABI 8, [2] before)
 * receives the slot class boundaries the forward's tile stage schedules by:
 * class_split[0] = 1 + the last slot that is a hub or has more than 6
 * messages, class_split[1] = 1 + the last slot that is a hub or has more than
 * 1 message, class_split[2] = 1 + the last slot that is a hub or has more
 * than 3 messages, class_split[3] = 1 + the last slot that is a hub or has
 * more than 7 messages (0 when there is none).  Slots past class_split[0]
 * (fp32 x) or class_split[3] (bf16 x) are "light" (2..6 / 2..7 messages),
 * slots past class_split[2] "short light" (at most 3: their own kernel
 * instance), slots past class_split[1] "lone" (self loop only).  Correct for
 * ANY order: an order that is not degree-sorted only moves the boundaries
 * towards num_dst. */
gfd_status gfd_plan_desc(const int32_t* rowptr, const int32_t* col, int64_t num_dst,
                         const int32_t* order, const int32_t* hub_rank, int32_t* desc,
                         int32_t* slot_cols, int64_t* class_split, gfd_stream_t stream);

/* Per-time-step snapshots of a temporal graph, every step in one pass (config
 * C3; replaces the reference's create_temporal_subgraph, dataset.py:198-240,
 * called per step by create_temporal_dataloaders, dataloader.py:99-135).
 * Steps are t_first .. t_first + num_steps - 1 of time_step[N] (int64).
 *   node_perm[N]   nodes of step 0 in ascending id, then step 1, ...; nodes
 *                  outside the steps last; node_pos[N] its inverse;
 *   step_ptr[S+1]  offsets of each step's nodes in node_perm;
 *   sub_edge_index [2, E] (row stride E): the edges whose endpoints are both in
 *                  one step, grouped by step, original order inside a step,
 *                  global node ids; sub_edge_local (nullable) the same edges
 *                  with step-local ids (position in the step's node list);
 *   edge_ptr[S+1]  offsets of each step's edges (edge_ptr[S] = kept edges).
 * Validates indices (GFD_ERR_INDEX) and synchronises the stream once. */
size_t gfd_temporal_workspace_size(int64_t num_nodes, int64_t num_edges, int32_t num_steps);
gfd_status gfd_temporal_snapshots(const int64_t* time_step, int64_t num_nodes,
                                  const int64_t* edge_index, int64_t num_edges, int64_t t_first,
                                  int32_t num_steps, int32_t* node_perm, int32_t* node_pos,
                                  int64_t* step_ptr, int64_t* sub_edge_index,
                                  int64_t* sub_edge_local, int64_t* edge_ptr, void* ws,
                                  size_t ws_bytes, gfd_stream_t stream);

/* Neighbour sampling for mini-batch training (replaces PyG NeighborLoader,
 * dataloader.py:42-66: num_neighbors = fanouts[0..hops), batch_size seeds,
 * sampling without replacement).  Hop l draws, for every node of frontier l,
 * min(fanouts[l], in-degree) distinct in-neighbours (sources of edges into
 * it) uniformly (Floyd's algorithm, counter-based random numbers keyed by
 * (seed, hop, node, draw): deterministic per seed); new sources are appended
 * in order of first appearance and form frontier l + 1.  The graph is the
 * gfd_csr_from_coo CSR (its appended self loops are not sampled).
 *   host fanouts[hops] (each <= 64); seeds[num_seeds] distinct node ids;
 *   local_of[N] int32 scratch that must be all -1 (left all -1 on return);
 *   n_id[max_nodes] global ids of the subgraph's nodes (seeds first);
 *   level_ptr[hops + 2] node offsets per hop (level 0 = the seeds);
 *   edge_src / edge_dst / edge_id[max_edges]: sampled edges, local ids of the
 *   source and destination, and the edge's CSR position; edge_ptr[hops + 1].
 * max_nodes / max_edges from gfd_sample_bounds.  Synchronises once. */
gfd_status gfd_sample_bounds(int64_t num_nodes, int64_t num_seeds, const int32_t* fanouts,
                             int32_t num_hops, int64_t* max_nodes, int64_t* max_edges);
size_t gfd_sample_workspace_size(int64_t num_nodes, int64_t num_seeds, const int32_t* fanouts,
                                 int32_t num_hops);
gfd_status gfd_sample_neighbors(const int32_t* rowptr, const int32_t* col, int64_t num_nodes,
                                const int64_t* seeds, int64_t num_seeds, const int32_t* fanouts,
                                int32_t num_hops, uint64_t seed, int32_t* local_of, int64_t* n_id,
                                int64_t* level_ptr, int64_t* edge_src, int64_t* edge_dst,
                                int64_t* edge_id, int64_t* edge_ptr, void* ws, size_t ws_bytes,
                                gfd_stream_t stream);

/* ---------------------------------------------------------------------------
 * GATConv forward (PyG GATConv.forward, concat=False, add_self_loops=True,
 * bias=True; gat.py:80 / tgn.py:94):
 *   out[i] = mean_h sum_{j in N(i)} alpha_ijh (W_h x_j) + bias
 *   alpha_ijh = softmax_j(leaky_relu(s_jh + t_ih, slope))  (eps 1e-16)
 *   s = (x W^T) . att_src, t = (x W^T) . att_dst  per head.
 * Computed aggregate-then-project: z_ih = sum_j alpha_ijh x_j (fp32), then
 * out_i = sum_h W_h z_ih / H on MFMA -- x rows (F wide) are gathered, never
 * the 512-wide projected rows.
 * ------------------------------------------------------------------------- */

/* Packed weights (device bytes): folded logit vectors and MFMA fragments. */
size_t gfd_gat_packed_size(int in_features, int heads, int channels);

/* lin_src.weight [H*C, F] row-major, att_src/att_dst [H*C] (PyG [1,H,C]) -> packed
 * (fp16 hi/lo fragments of W / H and of Wbar = mean_h W_h, folded logit
 * vectors, power-of-two scales). */
gfd_status gfd_gat_pack_weights(const float* weight, const float* att_src, const float* att_dst,
                                int in_features, int heads, int channels, void* packed,
                                gfd_stream_t stream);

/* Per-node attention logits st[r, 0:H] = s_r, st[r, H:2H] = t_r for rows
 * r in [0, num_rows) of x (x may point at any row; x_stride in elements). */
gfd_status gfd_gat_logits(const void* x, int x_dtype, int64_t num_rows, int in_features,
                          int64_t x_stride, const void* packed, int heads, int channels,
                          float* st, gfd_stream_t stream);

/* Execution plan of one destination range (all device pointers; NULL plan =
 * identity order, no hubs).  Built once per graph by gfd_plan_order and
 * gfd_plan_hubs on the range's rowptr. */
typedef struct gfd_plan {
  const int32_t* row_order;     /* [num_dst] tile order, or NULL for 0..num_dst-1      */
  const int32_t* slot_desc;     /* [4*num_dst] gfd_plan_desc output, or NULL           */
  const int32_t* slot_cols;     /* [8*num_dst] gfd_plan_desc output, or NULL           */
  const int32_t* hub_rank;      /* [num_dst] -1 or hub index (NULL iff num_hubs == 0)  */
  const int32_t* hub_chunk;     /* [4*num_chunks] {hub, e_begin, e_end, dst}           */
  const int32_t* hub_chunk_ptr; /* [num_hubs + 1]                                      */
  const int32_t* hub_dst;       /* [num_hubs]                                          */
  const int64_t* class_split;   /* [4] gfd_plan_desc class boundaries, or NULL: every  */
                                /* slot runs the general tile kernel                   */
  int64_t num_hubs;
  int64_t num_chunks;
} gfd_plan;

/* Workspace for gfd_gat_aggregate / gfd_gat_fwd (device bytes). */
size_t gfd_gat_fwd_workspace_size(int64_t num_nodes, int64_t num_dst, int in_features, int heads,
                                  int channels, int64_t num_hubs, int64_t num_chunks);

/* Fused softmax-aggregate-project for destinations [dst_offset, dst_offset+num_dst)
 * whose CSR slice is rowptr[0..num_dst] (absolute positions into col); sources
 * are global rows of x (N rows, "halo resident"); st holds logits for all N
 * rows (gfd_gat_logits).  dropout_p > 0 applies dropout to alpha with a
 * counter-based mask keyed by (seed, CSR position, head) -- reproducible in the
 * backward.  out [num_dst, C]; stats (nullable) [num_dst, 2H] = per-head
 * softmax max and denominator (sum of exp, without the eps) for the backward.
 * ``stages`` selects GFD_STAGE_HUBS (chunk partials + merge into ws),
 * GFD_STAGE_TILES (the tile kernels of every destination class, reading the
 * merged hub rows from ws) or GFD_STAGE_ALL; split calls must pass the same ws.
 * The tile stage schedules destinations by the plan's classes: general (hub
 * rows, 7+ messages; bf16 x: 8+), light (2..6 messages, GFD_LIGHT_MAX in
 * gfd_common.h; bf16 x: 2..7, GFD_LIGHT_MAX_BF16), lone (self loop only). */
#define GFD_STAGE_HUBS 1
#define GFD_STAGE_TILES 2
#define GFD_STAGE_ALL 3
/* single tile classes (profiling splits; the union equals GFD_STAGE_TILES):
 * general (k_stream<general>, or k_fused for F > 168), light
 * (k_stream<light>), lone (k_lone; for rows that are not 16-B aligned the light
 * kernel takes the lone class, when GFD_STAGE_TILES_LONE is asked for) */
#define GFD_STAGE_TILES_GENERAL 4
#define GFD_STAGE_TILES_LIGHT 8
#define GFD_STAGE_TILES_LONE 16
gfd_status gfd_gat_aggregate(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                             int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                             int64_t num_dst, int64_t dst_offset, const float* st,
                             const void* packed, const float* bias, int heads, int channels,
                             float negative_slope, float dropout_p, uint64_t dropout_seed,
                             const gfd_plan* plan, int stages, float* out, float* stats, void* ws,
                             size_t ws_bytes, gfd_stream_t stream);

/* gfd_gat_logits plus max |x| over the given rows: xmax (nullable, one device
 * float) is combined with its current value by atomic max, so initialise it to
 * 0 and, for a row-sharded x, reduce it over the shards (max) before
 * gfd_gat_aggregate_ex.  Replaces the same PyG GATConv.forward step as
 * gfd_gat_logits. */
gfd_status gfd_gat_logits_ex(const void* x, int x_dtype, int64_t rows, int in_features,
                             int64_t x_stride, const void* packed, int heads, int channels,
                             float* st, float* xmax, gfd_stream_t stream);

/* gfd_gat_logits_ex over a whole graph (rows = destinations = num_nodes), or a
 * contiguous destination range (x advanced to its first row, num_nodes = its
 * length, rowptr = the range's rowptr: the destination-sharded exchange),
 * fused with the outputs of the destinations whose only message is their self loop
 * (rowptr[i+1] - rowptr[i] == 1): their softmax has one term, so PyG's
 * out_i = mean_h W_h x_i + bias, written to out[i] (and, with stats, their
 * softmax max leaky(s_i + t_i) and denominator 1).  Other rows of out are not
 * touched; follow with gfd_gat_aggregate_ex(stages = HUBS | TILES_GENERAL |
 * TILES_LIGHT), which then leaves the lone class alone.  No dropout (with
 * dropout alpha is not 1).  GFD_ERR_UNSUPPORTED when x's base or pitch is not
 * 4-element aligned or F > 192 (use gfd_gat_logits_ex and the LONE stage).
 * Replaces the same PyG GATConv.forward steps as gfd_gat_logits, plus the
 * propagate of the self-loop-only destinations. */
gfd_status gfd_gat_logits_lone(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                               int64_t x_stride, const void* packed, int heads, int channels,
                               const int32_t* rowptr, const float* bias, float negative_slope,
                               float* st, float* xmax, float* out, float* stats,
                               gfd_stream_t stream);

/* gfd_gat_aggregate with xmax (nullable) = max |x| over ALL rows of x.  Every
 * aggregated row is a convex combination of x rows (dropout: times 1/(1-p)),
 * so the tile stage then uses one power-of-two scale for every Z row instead
 * of a per-row max.  Precondition: *xmax >= max |x| over every row any
 * destination gathers (the logits pass over all rows, reduced over shards).
 * The single scale is taken only while max |x| <= 2^20; beyond that (heavy-
 * tailed features, where small rows would lose the lo term) the kernels fall
 * back to each row's own scale, so results stay within the fp32 tolerance. */
gfd_status gfd_gat_aggregate_ex(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                                int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                                int64_t num_dst, int64_t dst_offset, const float* st,
                                const float* xmax, const void* packed, const float* bias,
                                int heads, int channels, float negative_slope, float dropout_p,
                                uint64_t dropout_seed, const gfd_plan* plan, int stages,
                                float* out, float* stats, void* ws, size_t ws_bytes,
                                gfd_stream_t stream);

/* One-call GATConv forward over the whole graph (num_dst = N, offset 0):
 * pack weights + logits + aggregate.  st (nullable, [N, 2H]) receives the
 * logits; ws must hold gfd_gat_fwd_workspace_size(N, N, F, H, C, hubs, chunks). */
gfd_status gfd_gat_fwd(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                       int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                       const float* weight, const float* att_src, const float* att_dst,
                       const float* bias, int heads, int channels, float negative_slope,
                       float dropout_p, uint64_t dropout_seed, const gfd_plan* plan, float* out,
                       float* st, float* stats, void* ws, size_t ws_bytes, gfd_stream_t stream);

/* Inference epilogue of the reference layer body (gat.py:82-91 and tgn.py
 * :96-105 in eval mode: GATConv -> BatchNorm1d(running stats) -> ReLU ->
 * dropout(identity) -> residual), applied by the kernels that store each
 * output row, so the layer output is written once:
 *   y = (conv + bias) * scale_shift[n] + scale_shift[C + n]
 *   y = max(y, 0)                           if relu
 *   y += residual[i * residual_stride + n]  if residual (the layer input)
 * BatchNorm1d folds to scale = gamma / sqrt(running_var + eps) and
 * shift = beta - running_mean * scale. */
typedef struct gfd_epilogue {
  const float* scale_shift; /* device [2 * C] */
  int relu;
  const float* residual;    /* device [N, residual_stride] or NULL */
  int64_t residual_stride;
  /* ABI 4: the model head Linear(C, 1) (gat.py:94) folded into the store of
   * the last layer: head_out[i] = y_i . head_weight + head_bias[0] is written
   * INSTEAD of the output row y_i (out may then be NULL).  head_out NULL: no
   * head.  Plan-scheduled path only (F <= 168); GFD_ERR_UNSUPPORTED else. */
  const float* head_weight; /* device [C] */
  const float* head_bias;   /* device [1] or NULL */
  float* head_out;          /* device [rows] */
} gfd_epilogue;

/* gfd_gat_fwd followed by the epilogue (ep may be NULL = gfd_gat_fwd).  With
 * an epilogue, stats must be NULL and dropout_p 0 (inference only: training
 * needs the raw GATConv output for the BatchNorm batch statistics). */
gfd_status gfd_gat_fwd_ep(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                          int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                          const float* weight, const float* att_src, const float* att_dst,
                          const float* bias, int heads, int channels, float negative_slope,
                          float dropout_p, uint64_t dropout_seed, const gfd_plan* plan,
                          const gfd_epilogue* ep, float* out, float* st, float* stats, void* ws,
                          size_t ws_bytes, gfd_stream_t stream);

/* gfd_gat_fwd_ep with the weights already packed (gfd_gat_pack_weights; ABI
 * 6): an inference caller packs a layer's weights once and reuses them while
 * they do not change (evaluate.py:73-98 runs the same trained layers on every
 * batch), instead of the seven small pack launches per call. */
gfd_status gfd_gat_fwd_ep_packed(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                                 int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                                 const void* packed, const float* bias, int heads, int channels,
                                 float negative_slope, float dropout_p, uint64_t dropout_seed,
                                 const gfd_plan* plan, const gfd_epilogue* ep, float* out,
                                 float* st, float* stats, void* ws, size_t ws_bytes,
                                 gfd_stream_t stream);

/* TemporalGNN head (tgn.py:108-111): h_new = GRUCell(h, h0) with PyTorch's
 * gate order (r, z, n) and out = h_new W_out^T + b_out, one kernel (gate
 * pre-activations stay on chip; exact fp32 MFMA products).  h [rows, C] with
 * row stride h_stride (multiple of 4, 16-B aligned), w_ih / w_hh [3C, C],
 * b_ih / b_hh [3C] (nullable), h0 (nullable = zeros, the reference's call,
 * tgn.py:88-89), w_out [out_channels, C], b_out [out_channels] (nullable);
 * h_new [rows, C], out [rows, out_channels].  C = 64. */
gfd_status gfd_gru_head(const float* h, int64_t rows, int channels, int64_t h_stride,
                        const float* w_ih, const float* b_ih, const float* w_hh,
                        const float* b_hh, const float* h0, int64_t h0_stride,
                        const float* w_out, const float* b_out, int out_channels, float* h_new,
                        float* out, gfd_stream_t stream);

/* Training backward of the same head (autograd of tgn.py:108-111 at
 * loss.backward(), train.py:142), given grad_out [rows, out_channels] and
 * grad_hnew (nullable) [rows, C] = dL/dh_new: recomputes the gates exactly as
 * gfd_gru_head does and writes grad_h [rows, C] = gi W_ih, grad_h0 [rows, C]
 * (required when h0 != NULL) = gh W_hh + dL/dh' z, and the gate gradients
 * gates_i = [dr | dz | dn] and gates_h = [dr | dz | dn r] ([rows, 3C] each;
 * pre-activation gradients of the x side and the h side) for gfd_atb:
 * grad_W_ih = gates_i^T h, grad_b_ih = colsum(gates_i), grad_W_hh = gates_h^T
 * h0, grad_b_hh = colsum(gates_h), grad_W_out = grad_out^T h_new, grad_b_out
 * = colsum(grad_out).  Same alignment rules as gfd_gru_head (w_hh required). */
gfd_status gfd_gru_head_bwd(const float* h, int64_t rows, int channels, int64_t h_stride,
                            const float* w_ih, const float* b_ih, const float* w_hh,
                            const float* b_hh, const float* h0, int64_t h0_stride,
                            const float* w_out, int out_channels, const float* grad_out,
                            const float* grad_hnew, float* grad_h, float* grad_h0,
                            float* gates_i, float* gates_h, gfd_stream_t stream);

/* Weight gradient of a row-wise linear map: out[m][n] = sum_r A[r][m] B[r][n]
 * (m < M <= 192, n < 64; A row stride lda >= M, B row stride ldb >= 64) and
 * colsum[m] = sum_r A[r][m] (nullable), fp32 MFMA, deterministic (fixed-order
 * split over row slabs).  Replaces the autograd weight-gradient GEMMs of the
 * TGN head's GRUCell and Linear (tgn.py:108-111). */
size_t gfd_atb_workspace_size(int64_t rows, int m);
gfd_status gfd_atb(const float* A, int64_t lda, int m, const float* B, int64_t ldb, int64_t rows,
                   float* out, float* colsum, void* ws, size_t ws_bytes, gfd_stream_t stream);

/* gfd_gat_aggregate_ex followed by the inference epilogue (ep nullable); the
 * residual rows are indexed like out (destination dst_offset + i at row i).
 * The destination-sharded model forward (gfd.dist) runs every layer through
 * it. */
gfd_status gfd_gat_aggregate_ep(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                                int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                                int64_t num_dst, int64_t dst_offset, const float* st,
                                const float* xmax, const void* packed, const float* bias,
                                int heads, int channels, float negative_slope, float dropout_p,
                                uint64_t dropout_seed, const gfd_plan* plan, int stages,
                                const gfd_epilogue* ep, float* out, float* stats, void* ws,
                                size_t ws_bytes, gfd_stream_t stream);

/* The destination-sharded exchange's layout (ABI 4): the source logits s and
 * the destination logits t in separate tables, so a rank's all-gather of s
 * lands directly where the aggregation reads it (no scatter into an [N, 2H]
 * table between the collective and the kernels).
 *   s_log [num_nodes rows, s_stride >= H]: s_j of every node (global rows);
 *   t_log [num_dst rows, t_stride >= H]: t_i of destination dst_offset + i.
 * out row i (destination dst_offset + i) at out + i * out_stride (>= C): a
 * rank writes its rows straight into its block of the next exchange's table.
 * gfd_gat_aggregate_ep(st) equals this with s_log = st, t_log = st +
 * 16 dst_offset + H, both strides 16, out_stride C.  Replaces the same PyG GATConv.forward
 * steps as gfd_gat_aggregate_ex (gat.py:80). */
gfd_status gfd_gat_aggregate_split(const void* x, int x_dtype, int64_t num_nodes,
                                   int in_features, int64_t x_stride, const int32_t* rowptr,
                                   const int32_t* col, int64_t num_dst, int64_t dst_offset,
                                   const float* s_log, int64_t s_stride, const float* t_log,
                                   int64_t t_stride, const float* xmax, const void* packed,
                                   const float* bias, int heads, int channels,
                                   float negative_slope, float dropout_p, uint64_t dropout_seed,
                                   const gfd_plan* plan, int stages, const gfd_epilogue* ep,
                                   float* out, int64_t out_stride, float* stats, void* ws,
                                   size_t ws_bytes, gfd_stream_t stream);

/* gfd_gat_logits_lone writing s (row i at s_log + i s_stride) and t (t_log +
 * i t_stride) separately, lone output rows at out + i out_stride: a rank's own destination block writes its s rows
 * straight into its slot of the all-gathered [N, H] s table.  Replaces the
 * same PyG GATConv.forward steps as gfd_gat_logits_lone. */
gfd_status gfd_gat_logits_lone_split(const void* x, int x_dtype, int64_t num_nodes,
                                     int in_features, int64_t x_stride, const void* packed,
                                     int heads, int channels, const int32_t* rowptr,
                                     const float* bias, float negative_slope, float* s_log,
                                     int64_t s_stride, float* t_log, int64_t t_stride,
                                     float* xmax, float* out, int64_t out_stride, float* stats,
                                     gfd_stream_t stream);

/* ---------------------------------------------------------------------------
 * GATConv backward (autograd of the PyG dataflow at loss.backward(),
 * train.py:142).  Given grad_out [N, C], the forward's
 * st [N, 2H] and stats [N, 2H], writes grad_x [N, F] (nullable), grad_weight
 * [H*C, F], grad_att_src/grad_att_dst [H*C], grad_bias [C] (nullable); grad_out
 * contiguous and 16-B aligned.  All
 * outputs are overwritten (not accumulated); deterministic (no float atomics).
 * Like the forward it gathers x rows, never the projected rows: the attention
 * gradient is <W_h^T grad_out_i / H, x_j>.  ``plan`` is the forward's plan
 * (tile order + destination hub chunks; NULL = identity order, no hubs);
 * ``src_plan`` (nullable) is a gfd_plan_hubs split of the CSC ``colptr``
 * (source hubs; only its hub fields are read).  x may be fp32 or bf16.
 * ------------------------------------------------------------------------- */
size_t gfd_gat_bwd_workspace_size(int64_t num_nodes, int64_t num_messages, int in_features,
                                  int heads, int channels, int64_t num_hubs, int64_t num_chunks,
                                  int64_t num_src_chunks);

gfd_status gfd_gat_bwd(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                       int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                       const gfd_plan* plan, const int32_t* colptr, const int32_t* csc_dst,
                       const int32_t* csc_eid, const gfd_plan* src_plan, int64_t num_messages,
                       const float* weight, const float* att_src, const float* att_dst,
                       int heads, int channels, float negative_slope, float dropout_p,
                       uint64_t dropout_seed, const float* st, const float* stats,
                       const float* grad_out, float* grad_x, float* grad_weight,
                       float* grad_att_src, float* grad_att_dst, float* grad_bias, void* ws,
                       size_t ws_bytes, gfd_stream_t stream);

/* gfd_gat_bwd with the per-column maxima of |x| supplied (ABI 6): x_colmax
 * (nullable = computed inside, as gfd_gat_bwd does) is uint32 [in_features]
 * holding max_n |x[n][f]| as float bits, from gfd_x_colmax over the same x.
 * The grad_W GEMM scales each x column by a power of two from it.  A layer
 * input that stays the same across training steps (the first layer's
 * features, train.py:115-143) needs it once per version of x. */
gfd_status gfd_gat_bwd_ex(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                          int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                          const gfd_plan* plan, const int32_t* colptr, const int32_t* csc_dst,
                          const int32_t* csc_eid, const gfd_plan* src_plan,
                          int64_t num_messages, const float* weight, const float* att_src,
                          const float* att_dst, int heads, int channels, float negative_slope,
                          float dropout_p, uint64_t dropout_seed, const float* st,
                          const float* stats, const float* grad_out, float* grad_x,
                          float* grad_weight, float* grad_att_src, float* grad_att_dst,
                          float* grad_bias, const uint32_t* x_colmax, void* ws, size_t ws_bytes,
                          gfd_stream_t stream);

/* gfd_gat_bwd_ex with the backward's dataflow chosen by the caller (ABI 7;
 * the library reads no environment):
 *   GFD_BWD_DH       the source pass writes dh' rows, the grad_W' GEMM reads
 *                    them (the default of gfd_gat_bwd / gfd_gat_bwd_ex);
 *   GFD_BWD_FUSED8   the fused source pass + grad_W' GEMM (k_src_gw), 8-wave
 *   GFD_BWD_FUSED16  or 16-wave blocks, taken only when grad_x is NULL and
 *                    in_features <= 192 (otherwise the dh' path runs).
 * Any other mode: GFD_ERR_ARGUMENT.  Replaces the same reference interface as
 * gfd_gat_bwd (loss.backward(), train.py:142). */
enum { GFD_BWD_DH = 0, GFD_BWD_FUSED8 = 1, GFD_BWD_FUSED16 = 2 };
gfd_status gfd_gat_bwd_mode(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                            int64_t x_stride, const int32_t* rowptr, const int32_t* col,
                            const gfd_plan* plan, const int32_t* colptr, const int32_t* csc_dst,
                            const int32_t* csc_eid, const gfd_plan* src_plan,
                            int64_t num_messages, const float* weight, const float* att_src,
                            const float* att_dst, int heads, int channels, float negative_slope,
                            float dropout_p, uint64_t dropout_seed, const float* st,
                            const float* stats, const float* grad_out, float* grad_x,
                            float* grad_weight, float* grad_att_src, float* grad_att_dst,
                            float* grad_bias, const uint32_t* x_colmax, int mode, void* ws,
                            size_t ws_bytes, gfd_stream_t stream);

/* Per-column maxima of |x| over rows [0, num_nodes) as float bits into
 * colmax (uint32 [in_features], in_features <= 256), for gfd_gat_bwd_ex. */
gfd_status gfd_x_colmax(const void* x, int x_dtype, int64_t num_nodes, int in_features,
                        int64_t x_stride, uint32_t* colmax, gfd_stream_t stream);

/* ---------------------------------------------------------------------------
 * Training-mode layer body (gat.py:82-91, tgn.py:96-105):
 *   out = residual + dropout(relu(BatchNorm1d_train(y)))
 * y [N, 64] fp32 (the GATConv output), residual nullable (fp32 rows [N, 64]).
 * Batch statistics are reduced deterministically (two-level, fp64 partials);
 * mean / invstd [64] are written for the backward; running_mean / running_var
 * (nullable) are updated as torch.nn.BatchNorm1d does (unbiased variance,
 * ``momentum`` weight on the batch value).  gamma / beta nullable = identity
 * (the backward needs them).  Dropout is a counter-based mask of
 * (seed, row * 64 + channel), regenerated by the backward; keep = 1/(1-p).
 * gfd_bn_relu_bwd writes grad_y [N, 64] (the residual's gradient is grad_out
 * itself) and grad_gamma / grad_beta [64] (nullable).
 * ------------------------------------------------------------------------- */
size_t gfd_bn_workspace_size(void);

gfd_status gfd_bn_relu_fwd(const float* y, const float* residual, int64_t N, int channels,
                           const float* gamma, const float* beta, float eps, float momentum,
                           float* running_mean, float* running_var, int relu, float dropout_p,
                           uint64_t seed, float* out, float* mean, float* invstd, void* ws,
                           size_t ws_bytes, gfd_stream_t stream);

gfd_status gfd_bn_relu_bwd(const float* y, const float* grad_out, int64_t N, int channels,
                           const float* gamma, const float* beta, const float* mean,
                           const float* invstd, int relu, float dropout_p, uint64_t seed,
                           float* grad_y, float* grad_gamma, float* grad_beta, void* ws,
                           size_t ws_bytes, gfd_stream_t stream);

/* -------------------------------------------------------------------------
 * Sparse halo exchange between destination shards (gfd.dist.HaloPlan; the
 * reference has no multi-GPU path -- this is the north star's "RCCL halo
 * exchange" of per-node rows).  dst[dst_rows[i]] = src[src_rows[i]] for
 * i < n, rows of ``cols`` fp32 values, row strides in floats; either index
 * list may be NULL (identity).  Packs the rows a peer needs before the
 * all-to-all and scatters the received ones to their node rows after it.
 * GFD_ERR_UNSUPPORTED past 2^31 copied elements.
 * ------------------------------------------------------------------------- */
gfd_status gfd_rows_copy(const float* src, int64_t src_stride, const int32_t* src_rows,
                         float* dst, int64_t dst_stride, const int32_t* dst_rows, int64_t n,
                         int cols, gfd_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* GFD_H */
