"""Destination-sharded multi-GPU execution.

One process per GPU (``torch.distributed``, backend "nccl" = RCCL on ROCm).
Ownership is by DESTINATION node: every in-edge of a destination lives on its
owner, so the segment softmax and the aggregation are rank-local and only
source-side data crosses GPUs.  Shards are contiguous destination ranges
balanced by message count (prefix sum over in-degree).

Layer 0 keeps ``x`` halo-resident (every rank holds the rows its in-edges
reference; for a power-law graph that is nearly all of x).  Only the SOURCE
logits s_j cross GPUs (``exchange_logits``): each rank computes ``[s | t]`` for
its own destination block (whose t it is the only reader of) and exchanges
the s half (``[N, H]`` fp32: 32 B per node instead of the 664 B feature row --
the "halo" of the north star).  The fused aggregate-project kernels then run on
the local shard with no further communication.  Hidden layers exchange the
previous layer's ``[N, 64]`` output rows together with the next layer's s.
Every exchange is either the sparse halo exchange (``HaloPlan``: only the
rows a shard's messages read, one RCCL all-to-all; the default of bench.py
and model_forward_sharded) or an all-gather of every block (below).

Layout (the split logits ABI, gfd_gat_aggregate_split): every exchanged table
is laid out by node row, each rank's block where the all-gather puts it, so
the collective writes straight into the tensors the kernels read -- no scatter
or concatenation between a collective and the next kernel:
  * equal blocks (``balance="nodes"``): a ``[world * per, cols]`` table, rank
    r's rows at ``r * per``; the collective is one in-place
    ``all_gather_into_tensor`` (RCCL and gloo alike);
  * message-balanced (uneven) blocks: a ``[N, cols]`` table with rank r's rows
    at its destination range; RCCL gathers into the row views (uneven
    all-gather); gloo, which has no uneven all-gather, through a padded buffer.
A hidden layer's aggregation writes its output rows straight into the rank's
block of the next exchange's ``[rows, 72]`` table (output row stride 72), the
next layer's s of those rows lands in columns 64..71, and after the in-place
all-gather the next layer reads h = table[:, :64] and s = table[:, 64:72] as
strided views.
"""
from __future__ import annotations

from typing import List, Optional, Tuple

import torch


def edge_balanced_bounds(rowptr: torch.Tensor, parts: int) -> List[int]:
    """Destination boundaries b_0=0 < ... < b_P=N with ~equal messages per part."""
    n = rowptr.numel() - 1
    total = int(rowptr[-1].item())
    if parts <= 1 or n == 0:
        return [0, n]
    targets = torch.tensor([total * k // parts for k in range(1, parts)], dtype=rowptr.dtype,
                           device=rowptr.device)
    cuts = torch.searchsorted(rowptr, targets).clamp_(0, n).tolist()
    bounds = [0] + [int(c) for c in cuts] + [n]
    for k in range(1, len(bounds)):          # keep them monotone
        bounds[k] = max(bounds[k], bounds[k - 1])
    return bounds


# Per-destination time model of the forward's stages on one MI355X (ns; C4
# round-4 stage times over their classes: logits pass 2.1 ms / 10M rows,
# light 6.1 ms / 6.2M rows, general 2.9 ms / 15.4M messages, hubs 2.3 ms /
# 21.3M messages plus a light-like projection row): what ``balance="cost"``
# equalises across ranks.
COST_ROW_NS, COST_LIGHT_NS, COST_GEN_MSG_NS, COST_HUB_MSG_NS, COST_HUB_ROW_NS = \
    0.21, 0.98, 0.19, 0.108, 1.0


def destination_costs(rowptr: torch.Tensor) -> torch.Tensor:
    """Modelled forward time of every destination (float64, ns) from its
    in-degree (self loop included): lone (1 message) -- the logits pass only;
    light (2..6); general (7..128, per message); hubs (> 128, per message plus
    the projection row).  Thresholds as the plan's (gfd_common.h, graph.py)."""
    from .graph import HUB_THRESHOLD
    deg = (rowptr[1:] - rowptr[:-1]).to(torch.float64)
    cost = torch.full_like(deg, COST_ROW_NS)
    cost += torch.where((deg >= 2) & (deg <= 6), COST_LIGHT_NS, 0.0)
    cost += torch.where((deg > 6) & (deg <= HUB_THRESHOLD), COST_GEN_MSG_NS * deg, 0.0)
    cost += torch.where(deg > HUB_THRESHOLD, COST_HUB_MSG_NS * deg + COST_HUB_ROW_NS, 0.0)
    return cost


def cost_balanced_bounds(rowptr: torch.Tensor, parts: int) -> List[int]:
    """Destination boundaries with ~equal modelled time per part
    (``destination_costs``): the node blocks of a randomly permuted power-law
    graph are equal in rows but not in hub messages (C4 at 8 ranks: the hub
    stage 0.36-0.50 ms across equal node blocks)."""
    n = rowptr.numel() - 1
    if parts <= 1 or n == 0:
        return [0, n]
    pre = torch.cumsum(destination_costs(rowptr), 0)
    total = float(pre[-1].item())
    targets = torch.tensor([total * k / parts for k in range(1, parts)], dtype=pre.dtype,
                           device=pre.device)
    cuts = torch.searchsorted(pre, targets).add_(1).clamp_(0, n).tolist()
    bounds = [0] + [int(c) for c in cuts] + [n]
    for k in range(1, len(bounds)):
        bounds[k] = max(bounds[k], bounds[k - 1])
    return bounds


def node_bounds(n: int, parts: int) -> List[int]:
    """Equal contiguous node blocks, padded so every block has ceil(n/parts) rows."""
    per = (n + parts - 1) // parts
    return [min(n, k * per) for k in range(parts + 1)]


def all_gather_rows(local: torch.Tensor, n: int, parts: int, group=None) -> torch.Tensor:
    """All-gather equal node blocks (last block zero-padded) into ``[n, cols]``."""
    import torch.distributed as dist
    per = (n + parts - 1) // parts
    cols = local.size(1)
    if local.size(0) < per:
        pad = local.new_zeros((per - local.size(0), cols))
        local = torch.cat([local, pad])
    out = local.new_empty((per * parts, cols))
    dist.all_gather_into_tensor(out, local.contiguous(), group=group)
    return out[:n]


def shard_ranges(rowptr: torch.Tensor, rank: int, world: int) -> Tuple[int, int]:
    b = edge_balanced_bounds(rowptr, world)
    return b[rank], b[rank + 1]


class ShardSpec:
    """One rank's share of a destination-sharded layer.

    ``dst_lo:dst_hi`` -- the destinations (and so the CSR messages) this rank
    owns; their attention logits are this rank's share of the exchange.
    ``balance="cost"``: ranges balanced by the modelled forward time of their
    destinations (``cost_balanced_bounds``; for the halo exchange, which takes
    any ranges).  ``balance="messages"``: ranges balanced by message count (prefix sum over
    in-degree); ``"nodes"``: equal node blocks of ``per = ceil(N / world)``
    rows (last one shorter) -- on a graph with randomly permuted ids (C4) the
    message counts then differ by ~2.6 % at 8 ranks, the destination counts
    (what the light tile stage is bound by) not at all, and the exchange is a
    plain equal-block all-gather straight into a ``[world * per, 8]`` table.
    ``node_lo:node_hi`` -- the equal node block (the tests' per-rank logits
    blocks).
    """

    def __init__(self, rowptr: torch.Tensor, rank: int, world: int, balance: str = "messages"):
        n = rowptr.numel() - 1
        self.rank, self.world, self.num_nodes = rank, world, n
        if balance not in ("messages", "nodes", "cost"):
            raise ValueError(f"balance must be 'messages', 'nodes' or 'cost', got {balance!r}")
        self.balance = balance
        self.node_bounds = node_bounds(n, world)
        self.dst_bounds = (edge_balanced_bounds(rowptr, world) if balance == "messages"
                           else cost_balanced_bounds(rowptr, world) if balance == "cost"
                           else list(self.node_bounds))
        self.per = max(max(self.dst_bounds[r + 1] - self.dst_bounds[r] for r in range(world)), 1)
        self.dst_lo, self.dst_hi = self.dst_bounds[rank], self.dst_bounds[rank + 1]
        self.node_lo, self.node_hi = self.node_bounds[rank], self.node_bounds[rank + 1]

    def equal_blocks(self) -> bool:
        """Rank r's destinations start at r * per (the node-balanced layout)."""
        return all(self.dst_bounds[r] == r * self.per for r in range(self.world))

    def __repr__(self) -> str:
        return (f"ShardSpec(rank={self.rank}/{self.world}, dst=[{self.dst_lo},{self.dst_hi}), "
                f"nodes=[{self.node_lo},{self.node_hi}))")


class LogitsTable:
    """The attention logits a shard's aggregation reads (gfd_gat_aggregate_split):
    ``s`` -- source logits of every node, a ``[rows >= N, >= 8]`` view (row =
    node id, any row stride); ``t`` -- destination logits of the rank's own
    destinations, a ``[n_dst, >= 8]`` view (local rows)."""

    def __init__(self, s: torch.Tensor, t: torch.Tensor):
        self.s, self.t = s, t

    @classmethod
    def from_st(cls, st: torch.Tensor, spec: "ShardSpec") -> "LogitsTable":
        """Views of an ``[N, 16]`` (s | t) table: no copies."""
        return cls(st[:, :8], st[spec.dst_lo:spec.dst_hi, 8:])

    def st(self, spec: "ShardSpec") -> torch.Tensor:
        """An ``[N, 16]`` table (t rows set for the own destinations only): tests."""
        n = spec.num_nodes
        out = torch.zeros((n, 16), dtype=self.s.dtype, device=self.s.device)
        out[:, :8] = self.s[:n, :8]
        out[spec.dst_lo:spec.dst_hi, 8:] = self.t[:, :8]
        return out


def exchange_table(cols: int, spec: ShardSpec, device, dtype=torch.float32) -> torch.Tensor:
    """An exchange table laid out by ``spec`` (module docstring): rows
    ``world * per`` for equal blocks, else N."""
    rows = spec.world * spec.per if spec.equal_blocks() else spec.num_nodes
    return torch.empty((max(rows, spec.num_nodes, 1), cols), dtype=dtype, device=device)


def own_block(table: torch.Tensor, spec: ShardSpec) -> torch.Tensor:
    """The rank's rows of an exchange table (its destinations, in order)."""
    return table[spec.dst_lo:spec.dst_hi]


def gather_blocks(table: torch.Tensor, spec: ShardSpec, group=None) -> None:
    """All-gather every rank's block of ``table`` in place (each rank has
    written its own block; every row of the table is then valid).  Equal
    blocks: one ``all_gather_into_tensor`` over the ``[world * per]`` rows.
    Uneven: RCCL's uneven all-gather into the row views, or for gloo (no
    uneven all-gather) a padded buffer copied out."""
    if spec.world == 1:
        return
    import torch.distributed as dist
    b, per, w = spec.dst_bounds, spec.per, spec.world
    if spec.equal_blocks():
        dist.all_gather_into_tensor(table[:w * per], table[spec.rank * per:(spec.rank + 1) * per],
                                    group=group)
        return
    views = [table[b[r]:b[r + 1]] for r in range(w)]
    if dist.get_backend(group) != "gloo":
        dist.all_gather(views, views[spec.rank], group=group)
        return
    buf = table.new_zeros((per * w,) + tuple(table.shape[1:]))
    mine = buf[spec.rank * per:spec.rank * per + views[spec.rank].shape[0]]
    mine.copy_(views[spec.rank])
    dist.all_gather_into_tensor(buf, buf[spec.rank * per:(spec.rank + 1) * per].clone(),
                                group=group)
    for r in range(w):
        views[r].copy_(buf[r * per:r * per + views[r].shape[0]])


def rows_copy(src: torch.Tensor, src_rows: Optional[torch.Tensor], dst: torch.Tensor,
              dst_rows: Optional[torch.Tensor]) -> None:
    """``dst[dst_rows[i]] = src[src_rows[i]]`` for fp32 row views of equal width
    (either index list None = identity): gfd_rows_copy on the GPU; plain
    indexing for the CPU tensors of the gloo tests."""
    n = (src_rows.numel() if src_rows is not None
         else dst_rows.numel() if dst_rows is not None else src.size(0))
    if n == 0:
        return
    if not dst.is_cuda:
        v = src[src_rows.long()] if src_rows is not None else src[:n]
        if dst_rows is not None:
            dst[dst_rows.long()] = v
        else:
            dst[:n] = v
        return
    from . import _lib
    assert src.dtype == dst.dtype == torch.float32 and src.size(1) == dst.size(1)
    assert src.stride(1) == 1 and dst.stride(1) == 1
    _lib.call("gfd_rows_copy", src.data_ptr(), src.stride(0), _lib.ptr(src_rows),
              dst.data_ptr(), dst.stride(0), _lib.ptr(dst_rows), n, src.size(1),
              _lib.stream_handle(dst.device))


def halo_needs(col: torch.Tensor, spec: ShardSpec) -> Tuple[torch.Tensor, List[int]]:
    """The rows of other ranks that a shard's messages read: the sorted unique
    sources of ``col`` (the shard's CSR columns, global node ids) outside the
    rank's own destination block, as int32, and their count per owner rank
    (owner = the rank whose destination block, and so whose logits pass, holds
    the row).  Sorted ids are grouped by owner, the order the all-to-all
    delivers them in."""
    ids = torch.unique(col.to(torch.int64))
    ids = ids[(ids < spec.dst_lo) | (ids >= spec.dst_hi)]
    cuts = torch.tensor(spec.dst_bounds[1:-1], dtype=torch.int64, device=ids.device)
    owner = torch.bucketize(ids, cuts, right=True)
    counts = torch.bincount(owner, minlength=spec.world).tolist()
    return ids.to(torch.int32), [int(c) for c in counts]


class HaloPlan:
    """Sparse exchange of per-node rows between destination shards: each rank
    receives only the rows of other ranks its own messages read (its halo) and
    sends each peer the own rows that peer reads.  At C4 over 8 node blocks a
    rank reads ~1.9M of the 8.75M other nodes, so the per-step exchange of the
    source logits (32 B per row) receives ~63 MB per rank instead of the
    all-gather's 280 MB.

    ``recv_rows`` (int32, grouped by owner rank, ``recv_counts`` per rank) --
    node rows written by the exchange; ``send_rows`` (int32, grouped by peer,
    ``send_counts``) -- own node rows sent.  Built once per (graph, shard) by
    ``create`` (two all-to-alls of counts and ids); ``exchange(table)``:
    gfd_rows_copy pack -> RCCL ``all_to_all_single`` -> gfd_rows_copy scatter,
    straight into the node-row table the kernels read."""

    def __init__(self, recv_rows: torch.Tensor, recv_counts: List[int],
                 send_rows: torch.Tensor, send_counts: List[int]):
        self.recv_rows, self.recv_counts = recv_rows, list(recv_counts)
        self.send_rows, self.send_counts = send_rows, list(send_counts)
        self._bufs = {}

    @classmethod
    def create(cls, col: torch.Tensor, spec: ShardSpec, group=None) -> "HaloPlan":
        import torch.distributed as dist
        recv_rows, recv_counts = halo_needs(col, spec)
        dev = recv_rows.device
        cdev = torch.device("cpu") if dist.get_backend(group) == "gloo" else dev
        rc = torch.tensor(recv_counts, dtype=torch.int64, device=cdev)
        sc = torch.empty_like(rc)
        dist.all_to_all_single(sc, rc, group=group)
        send_counts = [int(c) for c in sc.tolist()]
        send = torch.empty(sum(send_counts), dtype=torch.int32, device=cdev)
        dist.all_to_all_single(send, recv_rows.to(cdev), output_split_sizes=send_counts,
                               input_split_sizes=recv_counts, group=group)
        return cls(recv_rows, recv_counts, send.to(dev), send_counts)

    def bytes_received(self, cols: int, esz: int = 4) -> int:
        return int(self.recv_rows.numel()) * cols * esz

    def split(self, spec: ShardSpec, parts: int = 2) -> List["HaloPlan"]:
        """The same exchange in ``parts`` phases by row range: phase k moves the
        rows in the k-th of ``parts`` sub-ranges ``lo + (hi - lo) * k // parts``
        of each owner's destination block, so an owner can send phase k as soon
        as its logits pass has written that sub-range (the rest of the pass runs
        under the collective).  Every row of the plan is in exactly one phase."""
        b = spec.dst_bounds

        def cuts(q):
            lo, hi = b[q], b[q + 1]
            return [lo + (hi - lo) * k // parts for k in range(parts + 1)]

        def split_groups(rows, counts, cut_of):
            out_rows = [[] for _ in range(parts)]
            out_counts = [[0] * len(counts) for _ in range(parts)]
            off = 0
            for g, c in enumerate(counts):
                seg = rows[off:off + c]
                off += c
                cs = torch.tensor(cut_of(g)[1:-1], dtype=seg.dtype, device=seg.device)
                pos = torch.searchsorted(seg, cs).tolist() if c else [0] * (parts - 1)
                edges = [0] + [int(v) for v in pos] + [c]
                for k in range(parts):
                    out_rows[k].append(seg[edges[k]:edges[k + 1]])
                    out_counts[k][g] = edges[k + 1] - edges[k]
            return [torch.cat(r) if r else rows[:0] for r in out_rows], out_counts

        rr, rc = split_groups(self.recv_rows, self.recv_counts, cuts)          # owner q's cuts
        sr, sc = split_groups(self.send_rows, self.send_counts,
                              lambda g: cuts(spec.rank))                       # own cuts
        return [HaloPlan(rr[k], rc[k], sr[k], sc[k]) for k in range(parts)]

    def _buf(self, key, rows, like: torch.Tensor) -> torch.Tensor:
        shape = (max(rows, 1), like.size(1))
        b = self._bufs.get(key)
        if b is None or b.shape != shape or b.device != like.device or b.dtype != like.dtype:
            b = torch.empty(shape, dtype=like.dtype, device=like.device)
            self._bufs[key] = b
        return b

    def exchange(self, table: torch.Tensor, group=None) -> None:
        """``table`` (``[rows >= N, cols]`` fp32 by node row, unit column stride,
        any row stride): the rank's own rows are valid; afterwards so are its
        halo rows.  Rows neither own nor halo are not written."""
        self.exchange_async(table, group)()

    def exchange_async(self, table: torch.Tensor, group=None):
        """``exchange`` split at the collective: packs the own rows and issues
        the all-to-all (RCCL: asynchronously, on its own stream, ordered after
        the pack); returns ``finish()``, which makes the current stream wait
        for it and scatters the received rows.  gloo (CPU tests, host-staged
        rehearsals): synchronous."""
        import torch.distributed as dist
        ns, nr = int(self.send_rows.numel()), int(self.recv_rows.numel())
        send = self._buf("send", ns, table)
        recv = self._buf("recv", nr, table)
        rows_copy(table, self.send_rows, send, None)
        work = None
        if table.is_cuda and dist.get_backend(group) == "gloo":   # rehearsal: host-staged
            rc = torch.empty((max(nr, 1), table.size(1)), dtype=table.dtype)
            dist.all_to_all_single(rc[:nr], send[:ns].cpu(), output_split_sizes=self.recv_counts,
                                   input_split_sizes=self.send_counts, group=group)
            recv[:nr].copy_(rc[:nr])
        elif table.is_cuda:
            work = dist.all_to_all_single(recv[:nr], send[:ns], output_split_sizes=self.recv_counts,
                                          input_split_sizes=self.send_counts, group=group,
                                          async_op=True)
        else:
            dist.all_to_all_single(recv[:nr], send[:ns], output_split_sizes=self.recv_counts,
                                   input_split_sizes=self.send_counts, group=group)

        def finish():
            if work is not None:
                work.wait()
            rows_copy(recv, None, table, self.recv_rows)
        return finish


def all_gather_v_rows(local: torch.Tensor, bounds: List[int], group=None) -> torch.Tensor:
    """All-gather uneven row blocks (``bounds[r]:bounds[r+1]`` from rank r) into
    a new ``[N, cols]`` tensor (the model's final outputs)."""
    import torch.distributed as dist
    world = len(bounds) - 1
    sizes = [bounds[r + 1] - bounds[r] for r in range(world)]
    per = max(max(sizes), 1)
    cols = local.size(1)
    buf = local.new_zeros((per, cols))
    if local.size(0):
        buf[:local.size(0)] = local
    out = local.new_empty((per * world, cols))
    dist.all_gather_into_tensor(out, buf, group=group)
    return torch.cat([out[r * per:r * per + sizes[r]] for r in range(world)])


def pack_weights(weight: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor) -> torch.Tensor:
    """fp16 hi/lo MFMA fragments + folded attention vectors (gfd_gat_pack_weights)."""
    from . import _lib
    from .nn import SUPPORTED_CHANNELS, SUPPORTED_HEADS
    lib = _lib.load()
    H, C = SUPPORTED_HEADS, SUPPORTED_CHANNELS
    F = weight.size(1)
    if weight.shape != (H * C, F):
        raise ValueError(f"weight must be [{H * C}, F], got {tuple(weight.shape)}")
    dev = weight.device
    packed = torch.empty(lib.gfd_gat_packed_size(F, H, C), dtype=torch.uint8, device=dev)
    _lib.call("gfd_gat_pack_weights", weight.contiguous().data_ptr(),
              att_src.contiguous().data_ptr(), att_dst.contiguous().data_ptr(), F, H, C,
              packed.data_ptr(), _lib.stream_handle(dev))
    return packed


def shard_logits(x: torch.Tensor, packed: torch.Tensor, spec: ShardSpec,
                 xmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``[node_hi - node_lo, 16]`` attention logits (s | t) of this rank's node block.
    ``xmax`` (optional one-float device tensor) accumulates max |x| over the block
    (atomic max: start it at 0, reduce it over ranks before the aggregation)."""
    return logits_rows(x, packed, spec.node_lo, spec.node_hi, xmax)


def logits_rows(x: torch.Tensor, packed: torch.Tensor, lo: int, hi: int,
                xmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``[hi - lo, 16]`` attention logits (s | t) of rows lo:hi of x
    (gfd_gat_logits_ex, any row stride); ``xmax`` (optional one-float device
    tensor) accumulates max |x| over those rows (atomic max)."""
    from . import _lib
    from .nn import SUPPORTED_CHANNELS, SUPPORTED_HEADS
    H, C = SUPPORTED_HEADS, SUPPORTED_CHANNELS
    out = torch.empty((max(hi - lo, 0), 2 * H), dtype=torch.float32, device=x.device)
    if hi > lo:
        _lib.call("gfd_gat_logits_ex", x[lo:].data_ptr(), _lib.x_dtype_code(x), hi - lo,
                  x.size(1), x.stride(0), packed.data_ptr(), H, C, out.data_ptr(),
                  _lib.ptr(xmax), _lib.stream_handle(x.device))
    return out


def exchange_logits(x: torch.Tensor, packed: torch.Tensor, spec: ShardSpec,
                    xmax: Optional[torch.Tensor] = None, group=None,
                    logits_fn=None, halo: Optional["HaloPlan"] = None) -> LogitsTable:
    """The logits a shard's aggregation reads: s of every node, t of the rank's
    destinations.  ONE logits pass per rank over its own destination block
    (the only rows whose t it reads), its s rows written into its block of an
    ``[rows, 8]`` exchange table, then one in-place all-gather of that table
    (``gather_blocks``: 32 B per node; half the bytes of gathering [s | t]).
    ``logits_fn(lo, hi)`` -> [hi - lo, 16] replaces the HIP logits (tests).
    ``halo``: exchange only the rows the shard reads (HaloPlan) instead of
    all-gathering every block; the other rows of ``s`` are then not set."""
    H = 8
    N = x.size(0)
    if logits_fn is None:
        def logits_fn(lo, hi):
            return logits_rows(x, packed, lo, hi, xmax)
    if spec.world == 1:
        st = logits_fn(0, N)
        return LogitsTable(st[:, :H], st[:, H:])
    blk = logits_fn(spec.dst_lo, spec.dst_hi)
    s_tab = exchange_table(H, spec, blk.device)
    own_block(s_tab, spec).copy_(blk[:, :H])
    if halo is not None:
        halo.exchange(s_tab, group)
    else:
        gather_blocks(s_tab, spec, group)
    return LogitsTable(s_tab, blk[:, H:])


def _aggregate(h, graph, table: LogitsTable, packed, bias, spec, negative_slope, xmax, ep, out):
    from . import _lib
    from .graph import _ws
    from .nn import SUPPORTED_CHANNELS, SUPPORTED_HEADS
    lib = _lib.load()
    H, C = SUPPORTED_HEADS, SUPPORTED_CHANNELS
    N, F = h.shape
    n_dst = spec.dst_hi - spec.dst_lo
    if out is None:
        out = torch.empty((n_dst, C), dtype=torch.float32, device=h.device)
    if out.shape != (n_dst, C) or out.stride(1) != 1:
        raise ValueError(f"out must be a [{n_dst}, {C}] view with unit column stride")
    if n_dst == 0:
        return out
    s, t = table.s, table.t
    if s.stride(1) != 1 or t.stride(1) != 1 or s.size(0) < N or t.size(0) < n_dst:
        raise ValueError("logits table: s [>= N, 8] and t [>= n_dst, 8] row views")
    shard = graph.shard(spec.dst_lo, spec.dst_hi)   # plan built once per range, cached
    plan = shard.plan
    ws = _ws(lib.gfd_gat_fwd_workspace_size(N, n_dst, F, H, C, plan.num_hubs, plan.num_chunks),
             h.device)
    _lib.call("gfd_gat_aggregate_split", h.data_ptr(), _lib.x_dtype_code(h), N, F, h.stride(0),
              shard.rowptr.data_ptr(), graph.col.data_ptr(), n_dst, spec.dst_lo, s.data_ptr(),
              s.stride(0), t.data_ptr(), t.stride(0), _lib.ptr(xmax), packed.data_ptr(),
              _lib.ptr(bias), H, C, float(negative_slope), 0.0, 0, plan.cstruct(), 3,
              _lib.ct.byref(ep) if ep is not None else None, out.data_ptr(), out.stride(0), None,
              ws.data_ptr(), ws.numel(), _lib.stream_handle(h.device))
    return out


def _as_table(st, spec) -> LogitsTable:
    return st if isinstance(st, LogitsTable) else LogitsTable.from_st(st, spec)


def shard_aggregate(x: torch.Tensor, graph, st, packed: torch.Tensor,
                    bias: Optional[torch.Tensor], spec: ShardSpec,
                    negative_slope: float = 0.2,
                    xmax: Optional[torch.Tensor] = None,
                    out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``[dst_hi - dst_lo, 64]`` outputs of this rank's destinations
    (gfd_gat_aggregate_split, hubs + tiles) given the logits (a LogitsTable,
    or an ``[N, 16]`` s | t table); with ``xmax`` = max |x| over all rows the
    tile stage uses one Z-row scale.  ``out``: an ``[n_dst, 64]`` view (any row
    stride) to write into -- the rank's block of the next exchange table."""
    return _aggregate(x, graph, _as_table(st, spec), packed, bias, spec, negative_slope, xmax,
                      None, out)


def gat_conv_sharded(x: torch.Tensor, graph, weight: torch.Tensor, att_src: torch.Tensor,
                     att_dst: torch.Tensor, bias: Optional[torch.Tensor], spec: ShardSpec,
                     negative_slope: float = 0.2, gather_output: bool = True,
                     group=None, exchange: str = "halo") -> torch.Tensor:
    """Destination-sharded GATConv forward (eval) on this rank's GPU.

    ``x`` is halo-resident (all N rows on every rank, row stride may be
    padded), ``graph`` the full CSR.  Steps: pack weights -> ``exchange_logits``
    (the own block's logits, one in-place all-gather of the SOURCE logits
    ``[N, 8]``) and max|x| reduced -> fused aggregate-project over the rank's
    destinations -> (optionally) all-gather of the ``[n_dst, 64]`` outputs.
    ``exchange="halo"`` (default): the source logits by the sparse exchange
    (only the rows the shard reads; the plan cached on the graph).
    """
    if x.stride(1) != 1:
        raise ValueError("x rows must be contiguous")
    if exchange not in ("halo", "allgather"):
        raise ValueError(f"exchange must be 'halo' or 'allgather', got {exchange!r}")
    packed = pack_weights(weight, att_src, att_dst)
    xmax = torch.zeros(1, dtype=torch.float32, device=x.device)
    halo = halo_plan(graph, spec, group) if exchange == "halo" and spec.world > 1 else None
    table = exchange_logits(x, packed, spec, xmax, group=group, halo=halo)
    if spec.world > 1:
        import torch.distributed as dist
        dist.all_reduce(xmax, op=dist.ReduceOp.MAX, group=group)
    if not gather_output or spec.world == 1:
        return shard_aggregate(x, graph, table, packed, bias, spec, negative_slope, xmax)
    full = exchange_table(64, spec, x.device)
    shard_aggregate(x, graph, table, packed, bias, spec, negative_slope, xmax,
                    out=own_block(full, spec))
    gather_blocks(full, spec, group)
    return full[:spec.num_nodes]


# ---------------------------------------------------------------------------
# Model-level sharding: every layer of the reference stack (gat.py:79-94,
# tgn.py:93-111) destination-sharded, eval mode.

HID = 72   # hidden exchange row: h (64) | next layer's s (8)


def shard_aggregate_ep(h: torch.Tensor, graph, st, packed: torch.Tensor,
                       bias: Optional[torch.Tensor], spec: ShardSpec, negative_slope: float,
                       xmax: Optional[torch.Tensor], scale_shift: torch.Tensor, relu: bool,
                       residual: Optional[torch.Tensor],
                       out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """shard_aggregate with the layer body's inference epilogue fused into the
    output store (BN(eval) affine, ReLU, residual rows: ``residual`` = the
    layer input rows of this shard's destinations, any row stride).  ``out``
    as shard_aggregate (the rank's block of the next exchange table)."""
    from . import _lib
    ep = _lib.GfdEpilogue(scale_shift.data_ptr(), 1 if relu else 0, _lib.ptr(residual),
                          residual.stride(0) if residual is not None else 0)
    return _aggregate(h, graph, _as_table(st, spec), packed, bias, spec, negative_slope, xmax,
                      ep, out)


def layer_forward_sharded(conv, bn, h: torch.Tensor, graph, spec: ShardSpec, residual: bool,
                          group=None, st=None, xmax: Optional[torch.Tensor] = None,
                          packed: Optional[torch.Tensor] = None,
                          out: Optional[torch.Tensor] = None,
                          halo: Optional["HaloPlan"] = None) -> torch.Tensor:
    """One layer body on this rank: source logits exchanged
    (``exchange_logits``) and max|x| reduced, the rank's destinations
    aggregated with BN / ReLU / residual in the store.  ``h`` is the layer
    input for ALL N nodes (layer 0: the halo-resident features; hidden layers:
    the gathered table's view).  ``st`` / ``xmax`` / ``packed``: the logits
    table, max |h| and the packed weights when the caller already has them
    (hidden layers: they come with the gathered rows).  ``out``: where the
    output rows go (the rank's block of the next exchange table).  ``halo``:
    the source logits by the sparse exchange (exchange_logits)."""
    import torch.distributed as dist
    from .fused import bn_affine
    if packed is None:
        packed = pack_weights(conv.lin_src.weight.detach(), conv.att_src.detach(),
                              conv.att_dst.detach())
    if st is None:
        xmax = torch.zeros(1, dtype=torch.float32, device=h.device)
        st = exchange_logits(h, packed, spec, xmax, group=group, halo=halo)
        if spec.world > 1:
            dist.all_reduce(xmax, op=dist.ReduceOp.MAX, group=group)
    res = None
    if residual:
        res = h[spec.dst_lo:spec.dst_hi]
        res = res if res.dtype == torch.float32 else res.float()
    bias = conv.bias.detach() if conv.bias is not None else None
    return shard_aggregate_ep(h, graph, st, packed, bias, spec, conv.negative_slope, xmax,
                              bn_affine(bn, h.device), True, res, out=out)


def gather_hidden(table: torch.Tensor, next_conv, spec: ShardSpec, group=None,
                  halo: Optional["HaloPlan"] = None):
    """The exchange before a hidden layer, copy-free.  ``table`` is the
    ``[rows, 72]`` exchange table whose own block's columns 0..63 already hold
    this rank's output rows (the aggregation wrote them there).  The rank
    computes the next layer's logits of those rows (they are local), writes
    their s into columns 64..71 of its block, and ONE in-place all-gather
    fills every block; max |h| is reduced alongside.  Returns (h: [N, 64] view
    of the table, row stride 72; the LogitsTable: s = [N, 8] view of the
    table, t = this rank's destinations; max |h|; the packed weights).
    ``halo``: only the rows the shard reads are exchanged (72 floats each)."""
    import torch.distributed as dist
    H, C = 8, 64
    dev = table.device
    packed = pack_weights(next_conv.lin_src.weight.detach(), next_conv.att_src.detach(),
                          next_conv.att_dst.detach())
    mine = own_block(table, spec)
    n_dst = mine.size(0)
    xmax = torch.zeros(1, dtype=torch.float32, device=dev)
    st_l = logits_rows(mine[:, :C], packed, 0, n_dst, xmax)
    if n_dst:
        mine[:, C:] = st_l[:, :H]
    if halo is not None:
        halo.exchange(table, group)
    else:
        gather_blocks(table, spec, group)
    if spec.world > 1:
        dist.all_reduce(xmax, op=dist.ReduceOp.MAX, group=group)
    n = spec.num_nodes
    return table[:n, :C], LogitsTable(table[:n, C:], st_l[:, H:]), xmax, packed


class _SubSpec:
    """Destinations [lo, hi) of a rank's block, as _aggregate reads a spec."""

    def __init__(self, spec: ShardSpec, lo: int, hi: int):
        self.rank, self.world, self.num_nodes = spec.rank, spec.world, spec.num_nodes
        self.dst_lo, self.dst_hi = lo, hi


def layer_forward_gather_overlapped(conv, bn, h: torch.Tensor, graph, spec: ShardSpec,
                                    residual: bool, group, st, xmax, packed,
                                    table: torch.Tensor, next_conv, chunks: int = 4):
    """A hidden layer body fused with the exchange before the next layer, the
    collective overlapped with the aggregation (SURVEY.md §8e "Expected
    scaling"; equal node blocks).  The rank's destinations go in ``chunks``
    pieces: piece c is aggregated into its rows of the ``[rows, 72]`` exchange
    table, the next layer's logits of those rows are computed (s into columns
    64..71), and piece c of EVERY rank is all-gathered asynchronously (RCCL's
    own stream) while piece c + 1 is aggregated on the compute stream; every
    piece's collective is waited for at the end.  Returns what gather_hidden
    returns.  Same values as layer_forward_sharded + gather_hidden: the pieces
    are the same rows through the same kernels."""
    import torch.distributed as dist
    from .fused import bn_affine
    H, C = 8, 64
    dev = h.device
    if packed is None:
        packed = pack_weights(conv.lin_src.weight.detach(), conv.att_src.detach(),
                              conv.att_dst.detach())
    if st is None:
        xmax = torch.zeros(1, dtype=torch.float32, device=dev)
        st = exchange_logits(h, packed, spec, xmax, group=group)
        dist.all_reduce(xmax, op=dist.ReduceOp.MAX, group=group)
    st = _as_table(st, spec)
    next_packed = pack_weights(next_conv.lin_src.weight.detach(), next_conv.att_src.detach(),
                               next_conv.att_dst.detach())
    bias = conv.bias.detach() if conv.bias is not None else None
    aff = bn_affine(bn, dev)
    per, w, r = spec.per, spec.world, spec.rank
    n_own = spec.dst_hi - spec.dst_lo
    cs = max((per + chunks - 1) // chunks, 1)
    next_xmax = torch.zeros(1, dtype=torch.float32, device=dev)
    st_own = torch.empty((max(n_own, 0), 2 * H), dtype=torch.float32, device=dev)
    works = []
    for c0 in range(0, per, cs):
        c1 = min(c0 + cs, per)
        lo, hi = min(spec.dst_lo + c0, spec.dst_hi), min(spec.dst_lo + c1, spec.dst_hi)
        if hi > lo:   # the last rank's block may end before its padded rows
            sub = _SubSpec(spec, lo, hi)
            res = None
            if residual:
                res = h[lo:hi]
                res = res if res.dtype == torch.float32 else res.float()
            piece = table[lo:hi]
            shard_aggregate_ep(h, graph, LogitsTable(st.s, st.t[lo - spec.dst_lo:hi - spec.dst_lo]),
                               packed, bias, sub, conv.negative_slope, xmax, aff, True, res,
                               out=piece[:, :C])
            st_l = logits_rows(piece[:, :C], next_packed, 0, hi - lo, next_xmax)
            piece[:, C:] = st_l[:, :H]
            st_own[lo - spec.dst_lo:hi - spec.dst_lo] = st_l
        views = [table[q * per + c0:q * per + c1] for q in range(w)]
        works.append(dist.all_gather(views, views[r], group=group, async_op=True))
    for wk in works:
        wk.wait()
    dist.all_reduce(next_xmax, op=dist.ReduceOp.MAX, group=group)
    n = spec.num_nodes
    return table[:n, :C], LogitsTable(table[:n, C:], st_own[:, H:]), next_xmax, next_packed


def shard_columns(graph, spec: ShardSpec) -> torch.Tensor:
    """The CSR columns (global source ids) of the shard's messages; ``graph`` a
    CSRGraph or a ``(rowptr, col)`` pair."""
    rowptr, col = (graph.rowptr, graph.col) if hasattr(graph, "col") else graph
    return col[int(rowptr[spec.dst_lo]):int(rowptr[spec.dst_hi])]


def _group_key(group):
    """A process group by what the halo plan depends on -- its backend and
    member ranks -- not by ``id()``, which a destroyed group's successor may
    reuse."""
    import torch.distributed as dist
    g = group if group is not None else dist.group.WORLD
    try:
        ranks = tuple(dist.get_process_group_ranks(g))
    except Exception:  # noqa: BLE001 -- older torch: world size and rank only
        ranks = (dist.get_world_size(group), dist.get_rank(group))
    return (str(dist.get_backend(group)), ranks)


def halo_plan(graph, spec: ShardSpec, group=None) -> "HaloPlan":
    """The shard's HaloPlan, built once per (graph, destination range, world,
    process group membership) and cached on a CSRGraph (a ``(rowptr, col)``
    pair: built every call)."""
    key = (spec.dst_lo, spec.dst_hi, spec.world, spec.rank, _group_key(group))
    cache = getattr(graph, "_halo", None) if hasattr(graph, "_shards") else None
    if cache is not None and key in cache:
        return cache[key]
    plan = HaloPlan.create(shard_columns(graph, spec), spec, group)
    if hasattr(graph, "_shards"):
        if cache is None:
            cache = {}
            graph._halo = cache
        cache[key] = plan
    return plan


def model_forward_sharded(model, x: torch.Tensor, graph, spec: ShardSpec, group=None,
                          gather_output: bool = True, overlap_chunks: int = 4,
                          exchange: str = "halo"):
    """Destination-sharded eval forward of gfd.models.GAT / TemporalGNN (the
    reference's 2-3 layer stacks, gat.py:60-96, tgn.py:67-113) on this rank.

    Layer 0 reads the halo-resident features (all N rows on every rank; the
    exchange is the [N, 8] source-logits all-gather).  Every hidden layer's
    aggregation writes its rows straight into the rank's block of a ``[rows,
    72]`` exchange table, and ONE in-place collective (``gather_hidden``) moves
    them together with the next layer's source logits (computed by the row's
    owner): 2.9 GB in total at C4, no copies on either side of it.  The heads
    (Linear, GRUCell + Linear) are row-local.  ``exchange="halo"`` (default):
    every exchange moves only the rows the shard's messages read (HaloPlan,
    built once: ~22 % of the other ranks' rows at C4 over 8 ranks -- 0.6 GB
    instead of 2.9 GB per hidden layer); ``"allgather"``: the in-place
    all-gathers above, the hidden one in ``overlap_chunks`` pieces under the
    aggregation (equal blocks).  Returns the outputs of the rank's
    destinations, or of all N nodes (gather_output).  Inference only."""
    if model.training or torch.is_grad_enabled():
        raise RuntimeError("model_forward_sharded is inference-only: model.eval() and no_grad")
    if exchange not in ("halo", "allgather"):
        raise ValueError(f"exchange must be 'halo' or 'allgather', got {exchange!r}")
    h = x
    L = len(model.gat_layers)
    st = xmax = packed = None
    halo = halo_plan(graph, spec, group) if exchange == "halo" and spec.world > 1 else None
    for layer, conv in enumerate(model.gat_layers):
        bn = model.batch_norms[layer] if model.batch_norms is not None else None
        res = model.residual and h.size(-1) == model.hidden_channels
        if layer < L - 1 and spec.world > 1:
            table = exchange_table(HID, spec, x.device)
            nxt = model.gat_layers[layer + 1]
            if halo is None and spec.equal_blocks() and overlap_chunks > 1:
                # the all-gather under the compute
                h, st, xmax, packed = layer_forward_gather_overlapped(
                    conv, bn, h, graph, spec, res, group, st, xmax, packed, table, nxt,
                    overlap_chunks)
            else:
                layer_forward_sharded(conv, bn, h, graph, spec, res, group, st, xmax, packed,
                                      out=own_block(table, spec)[:, :64], halo=halo)
                h, st, xmax, packed = gather_hidden(table, nxt, spec, group, halo=halo)
        else:
            h = layer_forward_sharded(conv, bn, h, graph, spec, res, group, st, xmax, packed,
                                      halo=halo)
            st = xmax = packed = None
    if hasattr(model, "gru"):
        from .fused import gru_head
        out, hid = gru_head(model.gru, model.out, h)
        if gather_output and spec.world > 1:
            return (all_gather_v_rows(out, spec.dst_bounds, group=group),
                    all_gather_v_rows(hid, spec.dst_bounds, group=group))
        return out, hid
    out = model.out(h)
    if gather_output and spec.world > 1:
        return all_gather_v_rows(out, spec.dst_bounds, group=group)
    return out


# ---------------------------------------------------------------------------
# Sharded training (train.py:115-143 on the destination-sharded variant).
#
# Rank r owns destinations [lo, hi) and therefore every message into them
# (their segment softmax is rank-local).  Its share of a GATConv layer's
# forward AND backward runs on a LOCAL subgraph: the own destinations (rows
# 0 .. n_dst - 1, their CSR rows verbatim: input edges, self loop last) plus
# the sources those messages read from other blocks (rows n_dst ..; their
# only message is their own self loop, PyG's policy).  The local forward
# computes the halo rows' logits itself (x is resident on every rank: no
# exchange for layer 0) and the own rows' outputs exactly as the whole-graph
# forward does; the halo rows' outputs are not used, so their output
# gradient is zero and they add nothing to the backward, whose destination
# pass covers the own messages and whose source pass and grad_W' GEMM cover
# only the local rows -- the sources with local out-edges, not all N.  The
# parameter gradients of the ranks are partial sums of the whole-graph ones
# (every message belongs to exactly one rank), so ONE all-reduce of the
# layer's 0.35 MB of gradients completes them (``all_reduce_grads``).
# Dropout: the counter-based masks are keyed by CSR position, local here, so
# a sharded step draws different (equally distributed) masks than a
# single-process one.

class LocalGraph:
    """Rank-local subgraph of a destination shard (module section above).

    ``nodes`` -- int64 [N_loc] global id of each local row (own destinations
    ``lo .. hi - 1`` first, then the halo sources in ascending order);
    ``graph`` -- the local CSRGraph (PyG self-loop policy); ``n_dst``."""

    def __init__(self, nodes: torch.Tensor, graph, n_dst: int, lo: int, hi: int):
        self.nodes, self.graph, self.n_dst, self.lo, self.hi = nodes, graph, n_dst, lo, hi
        self._x_key = None
        self._x_loc = None

    @property
    def num_halo(self) -> int:
        return int(self.nodes.numel()) - self.n_dst

    def rows(self, x: torch.Tensor) -> torch.Tensor:
        """x's local rows (own block, then halo), through autograd when x
        requires grad; a constant x (layer 0's features) is gathered once per
        (storage, version) and kept."""
        if x.requires_grad:
            return x.index_select(0, self.nodes)
        key = (x.data_ptr(), x._version, tuple(x.shape), x.stride(0), x.dtype)
        if self._x_key != key:
            src = x if x.stride(1) == 1 else x.contiguous()
            self._x_loc = src.index_select(0, self.nodes)
            self._x_key = key
        return self._x_loc


def local_graph(graph, lo: int, hi: int) -> LocalGraph:
    """The LocalGraph of destinations [lo, hi) of ``graph`` (a CSRGraph on any
    device; CPU graphs serve the gloo tests).  Built once per range and cached
    on the graph (one host sync when built)."""
    cache = getattr(graph, "_local", None)
    key = (int(lo), int(hi))
    if cache is not None and key in cache:
        return cache[key]
    from .graph import CSRGraph
    rp = graph.rowptr
    dev = rp.device
    e0, e1 = int(rp[lo].item()), int(rp[hi].item())
    col = graph.col[e0:e1].to(torch.int64)
    n_dst = hi - lo
    halo = torch.unique(col[(col < lo) | (col >= hi)])          # sorted
    nodes = torch.cat([torch.arange(lo, hi, dtype=torch.int64, device=dev), halo])
    n_loc = int(nodes.numel())
    gmap = torch.full((graph.num_nodes,), -1, dtype=torch.int64, device=dev)
    gmap[nodes] = torch.arange(n_loc, dtype=torch.int64, device=dev)
    n_halo = n_loc - n_dst
    m_own = e1 - e0
    rowptr = torch.cat([rp[lo:hi + 1].to(torch.int64) - e0,
                        m_own + torch.arange(1, n_halo + 1, dtype=torch.int64, device=dev)])
    lcol = torch.cat([gmap[col], torch.arange(n_dst, n_loc, dtype=torch.int64, device=dev)])
    g = CSRGraph(n_loc, rowptr.to(torch.int32), lcol.to(torch.int32), m_own + n_halo,
                 m_own - n_dst)
    lg = LocalGraph(nodes, g, n_dst, lo, hi)
    if hasattr(graph, "_shards"):
        if cache is None:
            cache = {}
            graph._local = cache
        cache[key] = lg
    return lg


def gat_conv_local(x: torch.Tensor, local: LocalGraph, weight: torch.Tensor,
                   att_src: torch.Tensor, att_dst: torch.Tensor, bias: Optional[torch.Tensor],
                   negative_slope: float = 0.2, dropout: float = 0.0,
                   training: bool = False) -> torch.Tensor:
    """This rank's share of a GATConv forward with autograd: the ``[n_dst, 64]``
    outputs of its destinations, computed on the LocalGraph (gfd_gat_fwd /
    gfd_gat_bwd on the local rows).  After ``backward`` the parameter
    gradients hold this rank's partial sums: ``all_reduce_grads``."""
    from .nn import gat_conv
    out = gat_conv(local.rows(x), local.graph, weight, att_src, att_dst, bias,
                   negative_slope=negative_slope, dropout=dropout, training=training)
    return out[:local.n_dst]


def all_reduce_grads(params, group=None) -> None:
    """Sum the ranks' partial parameter gradients (one flat all-reduce; the
    reference layer's W, att_src, att_dst, bias: 0.35 MB at F = 166)."""
    import torch.distributed as dist
    ps = [p for p in params if p.requires_grad]
    if not ps or dist.get_world_size(group) == 1:
        return
    # every parameter in the same order on every rank, a missing gradient as
    # zeros (a rank whose shard never touched a parameter, set_to_none=True):
    # the flat buffers then line up element for element
    flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1)
                      for p in ps])
    dist.all_reduce(flat, group=group)
    off = 0
    for p in ps:
        n = p.numel()
        g = flat[off:off + n].view_as(p)
        if p.grad is None:
            p.grad = g.clone()
        else:
            p.grad.copy_(g)
        off += n


# ---------------------------------------------------------------------------
# Sharded training of the whole model (train.py:115-143 on destination shards)
#
# Layer 0 runs on the rank's LocalGraph with x gathered into the local order
# (``LocalGraph.rows``: x is a constant input, resident on every rank).  A
# hidden layer's input is the previous layer's output, which exists only on
# each node's owner: ``halo_rows`` brings the halo rows in (the HaloPlan of the
# shard: one all-to-all) and, in the backward, sends their gradients back to
# the owners (the reverse all-to-all), where they are added to the own rows'
# gradients -- so a hidden layer's grad_x crosses ranks exactly as its forward
# input did.  BatchNorm takes batch statistics over ALL nodes
# (``sharded_batch_norm``: the per-channel sums are all-reduced, forward and
# backward).  The loss is the reference's mean over labelled nodes, taken as
# each rank's sum over its own labelled nodes divided by the global count, so
# the ranks' losses add up to it; ``all_reduce_grads`` then sums the partial
# parameter gradients.


def _a2a(out: torch.Tensor, inp: torch.Tensor, out_splits, in_splits, group) -> None:
    """all_to_all_single of rows; device tensors over gloo (the one-GPU
    multi-process rehearsals) are staged through host memory."""
    import torch.distributed as dist
    if inp.is_cuda and dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        dist.all_to_all_single(o, inp.cpu(), output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=group)
        out.copy_(o)
    else:
        dist.all_to_all_single(out, inp, output_split_sizes=out_splits,
                               input_split_sizes=in_splits, group=group)


def _all_reduce(t: torch.Tensor, group) -> None:
    import torch.distributed as dist
    if t.is_cuda and dist.get_backend(group) == "gloo":
        h = t.cpu()
        dist.all_reduce(h, group=group)
        t.copy_(h)
    else:
        dist.all_reduce(t, group=group)


class _HaloRows(torch.autograd.Function):
    """own rows [n_own, C] -> local rows [n_own + n_halo, C] (LocalGraph order);
    backward: the halo rows' gradients back to their owners."""

    @staticmethod
    def forward(ctx, h_own, plan, lo, group):
        send_idx = plan.send_rows.to(h_own.device).long() - lo
        send = h_own.index_select(0, send_idx).contiguous()
        recv = h_own.new_empty((int(plan.recv_rows.numel()), h_own.size(1)))
        _a2a(recv, send, plan.recv_counts, plan.send_counts, group)
        ctx.plan, ctx.group, ctx.n_own = plan, group, h_own.size(0)
        ctx.save_for_backward(send_idx)
        return torch.cat([h_own, recv], 0)

    @staticmethod
    def backward(ctx, g_local):
        (send_idx,) = ctx.saved_tensors
        plan, n_own = ctx.plan, ctx.n_own
        g_own = g_local[:n_own].clone()
        g_halo = g_local[n_own:].contiguous()
        back = g_local.new_empty((int(send_idx.numel()), g_local.size(1)))
        _a2a(back, g_halo, plan.send_counts, plan.recv_counts, ctx.group)
        # one peer at a time: within a peer's list every own row appears once,
        # so each index_add is free of duplicate-index races and the peers are
        # added in a fixed order (deterministic)
        off = 0
        for c in plan.send_counts:
            if c:
                g_own.index_add_(0, send_idx[off:off + c], back[off:off + c])
            off += c
        return g_own, None, None, None


def halo_rows(h_own: torch.Tensor, plan: HaloPlan, lo: int, group=None) -> torch.Tensor:
    """[n_own + n_halo, C]: this rank's rows of a per-node tensor followed by its
    halo rows (ascending node id, as LocalGraph orders them), differentiable."""
    return _HaloRows.apply(h_own, plan, int(lo), group)


class _ShardedBN(torch.autograd.Function):
    """Training-mode BatchNorm1d over rows spread across ranks."""

    @staticmethod
    def forward(ctx, y, weight, bias, n_total, eps, group):
        # affine=False: weight 1, bias 0 (and no gradients for them)
        ctx.affine = weight is not None
        if weight is None:
            weight = torch.ones(y.size(1), dtype=y.dtype, device=y.device)
            bias = torch.zeros(y.size(1), dtype=y.dtype, device=y.device)
        yd = y.double()
        sums = torch.cat([yd.sum(0), (yd * yd).sum(0)])
        _all_reduce(sums, group)
        C = y.size(1)
        mean = sums[:C] / n_total
        var = (sums[C:] / n_total - mean * mean).clamp_min(0.0)
        invstd = (var + eps).rsqrt()
        xhat = ((yd - mean) * invstd).to(y.dtype)
        ctx.save_for_backward(xhat, weight, invstd.to(y.dtype))
        ctx.n_total, ctx.group = n_total, group
        mean, var = mean.to(y.dtype), var.to(y.dtype)
        ctx.mark_non_differentiable(mean, var)
        return xhat * weight + bias, mean, var

    @staticmethod
    def backward(ctx, g, _gm, _gv):
        xhat, weight, invstd = ctx.saved_tensors
        gd, xd = g.double(), xhat.double()
        sums = torch.cat([gd.sum(0), (gd * xd).sum(0)])
        grad_bias_part = sums[:g.size(1)].to(g.dtype).clone()     # this rank's partial sums
        grad_weight_part = sums[g.size(1):].to(g.dtype).clone()
        _all_reduce(sums, ctx.group)
        C, n = g.size(1), ctx.n_total
        dy = (weight.double() * invstd.double() / n) * (n * gd - sums[:C] - xd * sums[C:])
        if not ctx.affine:
            return dy.to(g.dtype), None, None, None, None, None
        return dy.to(g.dtype), grad_weight_part, grad_bias_part, None, None, None


def sharded_batch_norm(y: torch.Tensor, bn: torch.nn.BatchNorm1d, n_total: int,
                       group=None) -> torch.Tensor:
    """``bn(y)`` in training mode with the batch statistics of all ranks' rows
    (``n_total`` rows in all); the running statistics are updated as
    torch.nn.BatchNorm1d does (unbiased variance), identically on every rank.
    The weight / bias gradients are this rank's partial sums (all_reduce_grads)."""
    out, mean, var = _ShardedBN.apply(y, bn.weight, bn.bias, float(n_total), float(bn.eps), group)
    if bn.track_running_stats and bn.running_mean is not None:
        with torch.no_grad():
            bn.num_batches_tracked += 1
            m = bn.momentum if bn.momentum is not None else 1.0 / float(bn.num_batches_tracked)
            rdt = bn.running_mean.dtype
            unbiased = var.to(rdt) * (n_total / max(n_total - 1, 1))
            bn.running_mean.mul_(1 - m).add_(m * mean.to(rdt))
            bn.running_var.mul_(1 - m).add_(m * unbiased)
    return out


def gat_conv_on_local(conv, x_local: torch.Tensor, local: LocalGraph, training: bool):
    """One GATConv on the LocalGraph's rows (the HIP kernels); own rows returned."""
    from .nn import gat_conv
    out = gat_conv(x_local, local.graph, conv.lin_src.weight, conv.att_src, conv.att_dst,
                   conv.bias, conv.negative_slope, conv.dropout, training)
    return out[:local.n_dst]


def gat_forward_sharded_train(model, x: torch.Tensor, local: LocalGraph, plan: HaloPlan,
                              n_total: int, conv_fn=None, group=None) -> torch.Tensor:
    """The reference GAT's training forward (gat.py:60-96) for this rank's own
    nodes: [n_own, out] logits.  ``plan``: HaloPlan.create of the shard
    (hidden-layer halo exchange); ``n_total``: nodes over all ranks (BatchNorm);
    ``conv_fn(conv, x_local, local, training)``: the GATConv on local rows
    (default the HIP kernels; the CPU tests pass the oracle's arithmetic).
    Dropout masks are drawn per rank (equally distributed, not the
    single-process masks)."""
    import torch.nn.functional as F
    from .models import _head
    conv_fn = conv_fn or gat_conv_on_local
    lo = local.lo
    h_own = None
    for li, conv in enumerate(model.gat_layers):
        x_local = local.rows(x) if li == 0 else halo_rows(h_own, plan, lo, group)
        y = conv_fn(conv, x_local, local, model.training)
        if model.batch_norms is not None:
            bn = model.batch_norms[li]
            # eval: the running statistics, identical on every rank
            y = sharded_batch_norm(y, bn, n_total, group) if model.training else bn(y)
        y = F.dropout(F.relu(y), p=model.dropout, training=model.training)
        h_prev = x_local[:local.n_dst]
        h_own = h_prev + y if (model.residual and h_prev.size(-1) == y.size(-1)) else y
    return _head(model.out, h_own)
