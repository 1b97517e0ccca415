"""Destination-sharded multi-GPU execution.

One process per GPU (``torch.distributed``, backend "nccl" = RCCL on ROCm).
Ownership is by DESTINATION node: every in-edge of a destination lives on its
owner, so the segment softmax and the aggregation are rank-local and only
source-side data crosses GPUs.  Shards are contiguous destination ranges
balanced by message count (prefix sum over in-degree).

Layer 0 keeps ``x`` halo-resident (every rank holds the rows its in-edges
reference; for a power-law graph that is nearly all of x).  Only the SOURCE
logits s_j cross GPUs (``exchange_logits``): each rank computes ``[s | t]`` for
its own destination block (whose t it is the only reader of) and all-gathers
the s half (``[N, H]`` fp32: 32 B per node instead of the 664 B feature row --
the "halo" of the north star).  The fused aggregate-project kernels then run on the local shard
with no further communication.  Hidden layers all-gather the previous layer's
``[N, 64]`` output instead.
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
    ``balance="messages"``: ranges balanced by message count (prefix sum over
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
        if balance not in ("messages", "nodes"):
            raise ValueError(f"balance must be 'messages' or 'nodes', got {balance!r}")
        self.balance = balance
        self.node_bounds = node_bounds(n, world)
        self.dst_bounds = (edge_balanced_bounds(rowptr, world) if balance == "messages"
                           else list(self.node_bounds))
        self.per = max(max(self.dst_bounds[r + 1] - self.dst_bounds[r] for r in range(world)), 1)
        self.dst_lo, self.dst_hi = self.dst_bounds[rank], self.dst_bounds[rank + 1]
        self.node_lo, self.node_hi = self.node_bounds[rank], self.node_bounds[rank + 1]

    def __repr__(self) -> str:
        return (f"ShardSpec(rank={self.rank}/{self.world}, dst=[{self.dst_lo},{self.dst_hi}), "
                f"nodes=[{self.node_lo},{self.node_hi}))")


def all_gather_v_rows(local: torch.Tensor, bounds: List[int], group=None) -> torch.Tensor:
    """All-gather uneven row blocks (``bounds[r]:bounds[r+1]`` from rank r).

    RCCL's all-gather wants equal blocks, so each block is zero-padded to the
    largest one, gathered in one collective and the padding dropped."""
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
    (gfd_gat_logits_ex); ``xmax`` (optional one-float device tensor)
    accumulates max |x| over those rows (atomic max)."""
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
                    logits_fn=None) -> torch.Tensor:
    """The ``[N, 16]`` logits table a shard's aggregation reads: s (columns
    0..7) for every node, t (8..15) for the rank's destinations
    ``dst_lo:dst_hi`` (other rows' t are never read and left unset).

    ONE logits pass per rank, over its own destination block (the only rows
    whose t it reads), then one RCCL all-gather-v of the s half (``[N, 8]``:
    half the bytes of gathering [s | t]; blocks padded to the largest).
    ``logits_fn(lo, hi)`` -> [hi - lo, 16] replaces the HIP logits (tests)."""
    H = 8
    N = x.size(0)
    if logits_fn is None:
        def logits_fn(lo, hi):
            return logits_rows(x, packed, lo, hi, xmax)
    if spec.world == 1:
        return logits_fn(0, N)
    blk = logits_fn(spec.dst_lo, spec.dst_hi)
    s_all = all_gather_v_rows(blk[:, :H], spec.dst_bounds, group=group)
    st = torch.empty((N, 2 * H), dtype=torch.float32, device=blk.device)
    st[:, :H] = s_all
    if spec.dst_hi > spec.dst_lo:
        st[spec.dst_lo:spec.dst_hi, H:] = blk[:, H:]
    return st


def shard_aggregate(x: torch.Tensor, graph, st: torch.Tensor, packed: torch.Tensor,
                    bias: Optional[torch.Tensor], spec: ShardSpec,
                    negative_slope: float = 0.2,
                    xmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``[dst_hi - dst_lo, 64]`` outputs of this rank's destinations, given the
    all-gathered ``[N, 16]`` logits (gfd_gat_aggregate_ex, hubs + tiles); with
    ``xmax`` = max |x| over all rows the tile stage uses one Z-row scale."""
    from . import _lib
    from .graph import _ws
    from .nn import SUPPORTED_CHANNELS, SUPPORTED_HEADS
    lib = _lib.load()
    H, C = SUPPORTED_HEADS, SUPPORTED_CHANNELS
    N, F = x.shape
    n_dst = spec.dst_hi - spec.dst_lo
    out = torch.empty((n_dst, C), dtype=torch.float32, device=x.device)
    if n_dst == 0:
        return out
    shard = graph.shard(spec.dst_lo, spec.dst_hi)   # plan built once per range, cached
    plan = shard.plan
    ws = _ws(lib.gfd_gat_fwd_workspace_size(N, n_dst, F, H, C, plan.num_hubs, plan.num_chunks),
             x.device)
    _lib.call("gfd_gat_aggregate_ex", x.data_ptr(), _lib.x_dtype_code(x), N, F, x.stride(0),
              shard.rowptr.data_ptr(),
              graph.col.data_ptr(), n_dst, spec.dst_lo, st.data_ptr(), _lib.ptr(xmax),
              packed.data_ptr(),
              _lib.ptr(bias), H, C, float(negative_slope), 0.0, 0, plan.cstruct(),
              3, out.data_ptr(), None, ws.data_ptr(), ws.numel(), _lib.stream_handle(x.device))
    return out


def gat_conv_sharded(x: torch.Tensor, graph, weight: torch.Tensor, att_src: torch.Tensor,
                     att_dst: torch.Tensor, bias: Optional[torch.Tensor], spec: ShardSpec,
                     negative_slope: float = 0.2, gather_output: bool = True,
                     group=None) -> torch.Tensor:
    """Destination-sharded GATConv forward (eval) on this rank's GPU.

    ``x`` is halo-resident (all N rows on every rank, row stride may be
    padded), ``graph`` the full CSR.  Steps: pack weights -> ``exchange_logits``
    (one RCCL all-gather of the SOURCE logits ``[N, 8]``; t recomputed for the
    rank's own destinations) and max|x| reduced -> fused aggregate-project over
    the rank's destinations -> (optionally) all-gather-v of the ``[n_dst, 64]``
    outputs.
    """
    if x.stride(1) != 1:
        raise ValueError("x rows must be contiguous")
    packed = pack_weights(weight, att_src, att_dst)
    xmax = torch.zeros(1, dtype=torch.float32, device=x.device)
    st = exchange_logits(x, packed, spec, xmax, group=group)
    if spec.world > 1:
        import torch.distributed as dist
        dist.all_reduce(xmax, op=dist.ReduceOp.MAX, group=group)
    out = shard_aggregate(x, graph, st, packed, bias, spec, negative_slope, xmax)
    if gather_output:
        return all_gather_v_rows(out, spec.dst_bounds, group=group)
    return out


# ---------------------------------------------------------------------------
# Model-level sharding: every layer of the reference stack (gat.py:79-94,
# tgn.py:93-111) destination-sharded, eval mode.

def shard_aggregate_ep(h: torch.Tensor, graph, st: torch.Tensor, packed: torch.Tensor,
                       bias: Optional[torch.Tensor], spec: ShardSpec, negative_slope: float,
                       xmax: Optional[torch.Tensor], scale_shift: torch.Tensor, relu: bool,
                       residual: Optional[torch.Tensor]) -> torch.Tensor:
    """shard_aggregate with the layer body's inference epilogue fused into the
    output store (gfd_gat_aggregate_ep): BN(eval) affine, ReLU, residual rows
    (``residual`` = the layer input rows of this shard's destinations)."""
    from . import _lib
    from .graph import _ws
    from .nn import SUPPORTED_CHANNELS, SUPPORTED_HEADS
    lib = _lib.load()
    H, C = SUPPORTED_HEADS, SUPPORTED_CHANNELS
    N, F = h.shape
    n_dst = spec.dst_hi - spec.dst_lo
    out = torch.empty((n_dst, C), dtype=torch.float32, device=h.device)
    if n_dst == 0:
        return out
    shard = graph.shard(spec.dst_lo, spec.dst_hi)
    plan = shard.plan
    ws = _ws(lib.gfd_gat_fwd_workspace_size(N, n_dst, F, H, C, plan.num_hubs, plan.num_chunks),
             h.device)
    ep = _lib.GfdEpilogue(scale_shift.data_ptr(), 1 if relu else 0, _lib.ptr(residual),
                          residual.stride(0) if residual is not None else 0)
    _lib.call("gfd_gat_aggregate_ep", h.data_ptr(), _lib.x_dtype_code(h), N, F, h.stride(0),
              shard.rowptr.data_ptr(), graph.col.data_ptr(), n_dst, spec.dst_lo, st.data_ptr(),
              _lib.ptr(xmax), packed.data_ptr(), _lib.ptr(bias), H, C, float(negative_slope), 0.0,
              0, plan.cstruct(), 3, _lib.ct.byref(ep), out.data_ptr(), None, ws.data_ptr(),
              ws.numel(), _lib.stream_handle(h.device))
    return out


def layer_forward_sharded(conv, bn, h: torch.Tensor, graph, spec: ShardSpec, residual: bool,
                          group=None, st: Optional[torch.Tensor] = None,
                          xmax: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One layer body on this rank: source logits exchanged
    (``exchange_logits``) and max|x| reduced, the rank's destinations
    aggregated with BN / ReLU / residual in the store.  ``h`` is the layer
    input for ALL N nodes (layer 0: the halo-resident features).  ``st`` /
    ``xmax``: the logits table and max |h| when the caller already has them
    (hidden layers: they arrive with the all-gathered rows)."""
    import torch.distributed as dist
    from .fused import bn_affine
    packed = pack_weights(conv.lin_src.weight.detach(), conv.att_src.detach(),
                          conv.att_dst.detach())
    if st is None:
        xmax = torch.zeros(1, dtype=torch.float32, device=h.device)
        st = exchange_logits(h, packed, spec, xmax, group=group)
        if spec.world > 1:
            dist.all_reduce(xmax, op=dist.ReduceOp.MAX, group=group)
    res = None
    if residual:
        res = h[spec.dst_lo:spec.dst_hi]
        res = res if res.dtype == torch.float32 else res.float()
    bias = conv.bias.detach() if conv.bias is not None else None
    return shard_aggregate_ep(h, graph, st, packed, bias, spec, conv.negative_slope, xmax,
                              bn_affine(bn, h.device), True, res)


def gather_hidden(out_local: torch.Tensor, next_conv, spec: ShardSpec, group=None):
    """The exchange before a hidden layer, as ONE collective: every rank
    computes the next layer's logits [s | t] of its own output rows (they are
    local), then all-gathers ``[out | s | max|out|]`` rows (all-gather-v,
    72 columns).  Returns (h [N, 64] view with row stride 72, the [N, 16]
    logits table -- s for every node, t for this rank's destinations -- and
    max |h| over all rows, reduced over ranks by the same collective)."""
    H, C = 8, 64
    n_dst = out_local.size(0)
    dev = out_local.device
    packed = pack_weights(next_conv.lin_src.weight.detach(), next_conv.att_src.detach(),
                          next_conv.att_dst.detach())
    xmax_l = torch.zeros(1, dtype=torch.float32, device=dev)
    st_l = logits_rows(out_local, packed, 0, n_dst, xmax_l)
    rows = torch.empty((n_dst, C + H), dtype=torch.float32, device=dev)
    rows[:, :C] = out_local
    rows[:, C:] = st_l[:, :H]
    # max |h| travels in an extra column of each rank's first row block: the
    # padded row 0 of every block (all_gather_v pads to the largest block)
    world = spec.world
    sizes = [spec.dst_bounds[r + 1] - spec.dst_bounds[r] for r in range(world)]
    per = max(max(sizes), 1) + 1
    import torch.distributed as dist
    buf = rows.new_zeros((per, C + H))
    buf[0, 0] = xmax_l[0]
    if n_dst:
        buf[1:1 + n_dst] = rows
    allb = rows.new_empty((per * world, C + H))
    dist.all_gather_into_tensor(allb, buf, group=group)
    xmax = allb[0::per, 0].max().reshape(1).contiguous()
    full = torch.cat([allb[r * per + 1:r * per + 1 + sizes[r]] for r in range(world)])
    st = torch.empty((full.size(0), 2 * H), dtype=torch.float32, device=dev)
    st[:, :H] = full[:, C:]
    if n_dst:
        st[spec.dst_lo:spec.dst_hi, H:] = st_l[:, H:]
    return full[:, :C], st, xmax


def model_forward_sharded(model, x: torch.Tensor, graph, spec: ShardSpec, group=None,
                          gather_output: bool = True):
    """Destination-sharded eval forward of gfd.models.GAT / TemporalGNN (the
    reference's 2-3 layer stacks, gat.py:60-96, tgn.py:67-113) on this rank.

    Layer 0 reads the halo-resident features (all N rows on every rank; the
    exchange is the [N, 8] source-logits all-gather).  Before each layer >= 1
    ONE collective (``gather_hidden``) moves the previous layer's output rows
    together with the next layer's source logits, computed by the row's owner
    (72 columns: 2.9 GB in total at C4) -- the logits exchange rides along
    instead of costing a second collective.  The heads (Linear, GRUCell +
    Linear) are row-local.  Returns the outputs of the rank's destinations, or
    of all N nodes (gather_output).  Inference only."""
    if model.training or torch.is_grad_enabled():
        raise RuntimeError("model_forward_sharded is inference-only: model.eval() and no_grad")
    h = x
    L = len(model.gat_layers)
    st = xmax = None
    for layer, conv in enumerate(model.gat_layers):
        bn = model.batch_norms[layer] if model.batch_norms is not None else None
        res = model.residual and h.size(-1) == model.hidden_channels
        out_local = layer_forward_sharded(conv, bn, h, graph, spec, res, group, st, xmax)
        if layer < L - 1:
            if spec.world > 1:
                h, st, xmax = gather_hidden(out_local, model.gat_layers[layer + 1], spec, group)
            else:
                h, st, xmax = out_local, None, None
        else:
            h = out_local
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
