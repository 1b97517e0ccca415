"""CPU oracle for the GATConv hot path -- TEST INFRASTRUCTURE ONLY.

This module is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The product path (``gfd.nn.GATConv``) runs exclusively on the HIP library
and fails loudly when it is missing.

What it restates
----------------
The reference imports ``GATConv`` from the third-party PyTorch Geometric
package (``/root/reference/src/models/gat.py:4``, ``tgn.py:4``), constructs it as
``GATConv(in, 64, heads=8, concat=False, dropout=p)`` (gat.py:39,45,51;
tgn.py:43,49,55) and calls it as ``gat(h, edge_index)`` (gat.py:80, tgn.py:94).
PyG is NOT vendored in the reference and is not installed here
(``torch-geometric>=2.0.0``, unpinned: /root/reference/setup.py:13;
``torch-scatter>=2.0.9``: setup.py:14).  This file restates the published PyG
2.x algorithm for ``concat=False`` exactly as PyG's own CPU dataflow executes
it:

1. ``x_src = x_dst = lin_src(x).view(-1, H, C)``   (``lin_dst is lin_src``)
2. ``alpha_src = (x_src * att_src).sum(-1)``; ``alpha_dst`` likewise
3. ``remove_self_loops`` then ``add_self_loops`` (loops appended at the end,
   duplicates kept)
4. ``alpha = leaky_relu(alpha_src[j] + alpha_dst[i], 0.2)``
5. ``softmax(alpha, index=i)``: scatter-max, ``exp(a - max[i])``,
   scatter-sum, ``/ (sum + 1e-16)``
6. ``dropout(alpha, p)`` when training
7. message ``alpha[..., None] * x_src[j]``; scatter-add into ``i``
8. ``out.mean(dim=1) + bias``

Parity status: PyG itself cannot be imported here, so the *arithmetic* of this
restatement is pinned only against PyG's published algorithm (SURVEY.md §8c,
"parity unpinned vs real PyG").  The *model wiring* and the *weights* are
pinned: ``tests/golden/make_golden.py`` runs the reference's own
``src/models/gat.py`` / ``tgn.py`` with this class injected as
``torch_geometric.nn.GATConv`` and the shipped checkpoints loaded strictly.
"""
from __future__ import annotations

import math
from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

NEG_SLOPE = 0.2
SOFTMAX_EPS = 1e-16


def remove_then_add_self_loops(edge_index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG ``remove_self_loops`` + ``add_self_loops`` (loops appended last)."""
    mask = edge_index[0] != edge_index[1]
    kept = edge_index[:, mask]
    loops = torch.arange(num_nodes, dtype=edge_index.dtype, device=edge_index.device)
    return torch.cat([kept, torch.stack([loops, loops])], dim=1)


def segment_softmax(alpha: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """PyG ``utils.softmax`` over destination segments (``[E', H]``)."""
    H = alpha.size(1)
    amax = torch.full((num_nodes, H), -math.inf, dtype=alpha.dtype)
    amax = amax.scatter_reduce(0, index[:, None].expand(-1, H), alpha.detach(),
                               reduce="amax", include_self=True)
    out = (alpha - amax.index_select(0, index)).exp()
    ssum = torch.zeros((num_nodes, H), dtype=alpha.dtype).index_add(0, index, out)
    return out / (ssum.index_select(0, index) + SOFTMAX_EPS)


def gatconv_forward(x: torch.Tensor, edge_index: torch.Tensor, weight: torch.Tensor,
                    att_src: torch.Tensor, att_dst: torch.Tensor, bias: Optional[torch.Tensor],
                    heads: int = 8, negative_slope: float = NEG_SLOPE, dropout: float = 0.0,
                    training: bool = False, return_stats: bool = False,
                    alpha_mask: Optional[torch.Tensor] = None):
    """Functional PyG-dataflow GATConv (concat=False). Differentiable by autograd.

    ``weight`` is ``lin_src.weight`` ``[H*C, F]``; ``att_*`` are ``[1, H, C]``.
    With ``return_stats`` also returns the edge list with self loops, the
    per-(node, head) softmax max and sum, and the un-dropped alpha.
    ``alpha_mask`` ([E', H], already scaled by 1/(1-p)) replaces F.dropout so a
    test can impose the exact mask the device drew.
    """
    N = x.size(0)
    H = heads
    C = weight.size(0) // H
    h = (x @ weight.t()).view(N, H, C)                     # lin_src(x)
    a_src = (h * att_src).sum(-1)                          # [N, H]
    a_dst = (h * att_dst).sum(-1)
    ei = remove_then_add_self_loops(edge_index, N)
    j, i = ei[0], ei[1]
    logit = F.leaky_relu(a_src.index_select(0, j) + a_dst.index_select(0, i), negative_slope)
    alpha = segment_softmax(logit, i, N)
    alpha_d = alpha * alpha_mask if alpha_mask is not None else \
        F.dropout(alpha, p=dropout, training=training)
    msg = alpha_d.unsqueeze(-1) * h.index_select(0, j)     # [E', H, C]
    agg = torch.zeros((N, H, C), dtype=x.dtype).index_add(0, i, msg)
    out = agg.mean(dim=1)
    if bias is not None:
        out = out + bias
    if not return_stats:
        return out
    with torch.no_grad():
        amax = torch.full((N, H), -math.inf, dtype=x.dtype).scatter_reduce(
            0, i[:, None].expand(-1, H), logit, reduce="amax", include_self=True)
        ssum = torch.zeros((N, H), dtype=x.dtype).index_add(
            0, i, (logit - amax.index_select(0, i)).exp())
    return out, {"edge_index": ei, "alpha": alpha.detach(), "max": amax, "sum": ssum}


def gatconv_forward_chunked(x: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor,
                            weight: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor,
                            bias: torch.Tensor, heads: int = 8, chunk_edges: int = 4_000_000,
                            dst_range: Optional[Tuple[int, int]] = None) -> torch.Tensor:
    """Same math on a destination-sorted CSR (self loops already in), processed
    in destination chunks of at most ``chunk_edges`` messages so the PyG
    ``[E', H, C]`` message tensor stays bounded (SURVEY.md §8d CPU baseline).
    Used for the bench's bounded CPU-baseline sample; eval mode only."""
    N = x.size(0)
    H = heads
    C = weight.size(0) // H
    h = (x @ weight.t()).view(N, H, C)
    a_src = (h * att_src).sum(-1)
    a_dst = (h * att_dst).sum(-1)
    lo, hi = dst_range if dst_range is not None else (0, N)
    out = torch.empty((hi - lo, C), dtype=x.dtype)
    start = lo
    rp = rowptr
    while start < hi:
        # grow the chunk until it holds ~chunk_edges messages
        e0 = int(rp[start])
        # largest node k with rp[k] <= e0 + chunk_edges, clamped to [start+1, hi]
        k = int(torch.searchsorted(rp, torch.tensor([e0 + chunk_edges], dtype=rp.dtype),
                                   right=True).item()) - 1
        stop = min(hi, max(start + 1, k))
        e1 = int(rp[stop])
        j = col[e0:e1].long()
        seg = torch.repeat_interleave(torch.arange(stop - start), (rp[start + 1:stop + 1] - rp[start:stop]).long())
        i_glob = seg + start
        logit = F.leaky_relu(a_src.index_select(0, j) + a_dst.index_select(0, i_glob), NEG_SLOPE)
        alpha = segment_softmax(logit, seg, stop - start)
        msg = alpha.unsqueeze(-1) * h.index_select(0, j)
        agg = torch.zeros((stop - start, H, C), dtype=x.dtype).index_add(0, seg, msg)
        out[start - lo:stop - lo] = agg.mean(dim=1) + bias
        start = stop
    return out


def gatconv_forward_at(x: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor,
                       dsts: torch.Tensor, weight: torch.Tensor, att_src: torch.Tensor,
                       att_dst: torch.Tensor, bias: torch.Tensor, heads: int = 8) -> torch.Tensor:
    """PyG-dataflow outputs for the destinations ``dsts`` only (a CSR with self
    loops already in).  Projects just the rows those destinations touch, so it
    stays cheap on 10M-node graphs: the sampled full-size parity check."""
    H = heads
    C = weight.size(0) // H
    dsts = dsts.long()
    starts, ends = rowptr[dsts].long(), rowptr[dsts + 1].long()
    lens = ends - starts
    seg = torch.repeat_interleave(torch.arange(dsts.numel()), lens)
    pos = torch.repeat_interleave(starts - torch.cumsum(lens, 0) + lens, lens) + torch.arange(int(lens.sum()))
    j = col[pos].long()
    nodes, inv = torch.unique(torch.cat([j, dsts]), return_inverse=True)
    h = (x[nodes] @ weight.t()).view(-1, H, C)
    a_src = (h * att_src).sum(-1)
    a_dst = (h * att_dst).sum(-1)
    jl, il = inv[:j.numel()], inv[j.numel():]
    logit = F.leaky_relu(a_src[jl] + a_dst[il][seg], NEG_SLOPE)
    alpha = segment_softmax(logit, seg, dsts.numel())
    agg = torch.zeros((dsts.numel(), H, C), dtype=x.dtype).index_add(0, seg, alpha.unsqueeze(-1) * h[jl])
    return agg.mean(dim=1) + bias


class gatconv_forward_sampled:  # noqa: N801 (a namespace: prepare once, run many)
    """PyG-dataflow outputs for a destination sample of a (device) CSR, with
    only the rows the sample gathers copied to the host.  ``prepare`` builds
    the induced sub-problem (the rows of every source of the sampled
    destinations and of the destinations themselves, as fp32 on the CPU);
    ``run`` is the same dataflow as ``gatconv_forward_at``.  Used by the
    full-size parity tests (tests/test_bench_parity_gpu.py) and by bench.py's
    CPU-baseline leg."""

    @staticmethod
    def prepare(x: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor,
                dsts: torch.Tensor) -> dict:
        dsts = dsts.long()
        rp = rowptr.long()
        starts, ends = rp[dsts], rp[dsts + 1]
        lens = ends - starts
        seg = torch.repeat_interleave(torch.arange(dsts.numel(), device=dsts.device), lens)
        off = torch.cumsum(lens, 0) - lens
        pos = starts[seg] + torch.arange(int(lens.sum()), device=dsts.device) - off[seg]
        j = col[pos].long()
        nodes, inv = torch.unique(torch.cat([j, dsts]), return_inverse=True)
        return {"x": x[nodes].float().cpu(), "jl": inv[:j.numel()].cpu(),
                "il": inv[j.numel():].cpu(), "seg": seg.cpu(), "n": dsts.numel(),
                "rows": nodes.numel(), "dsts": dsts.cpu()}

    @staticmethod
    def prepare_indices(rowptr: torch.Tensor, col: torch.Tensor, dsts: torch.Tensor) -> dict:
        """``prepare`` without copying rows: the index arrays only (host), so
        ``run_from`` gathers the rows out of the full host feature matrix."""
        dsts = dsts.long()
        rp = rowptr.long()
        starts, ends = rp[dsts], rp[dsts + 1]
        lens = ends - starts
        seg = torch.repeat_interleave(torch.arange(dsts.numel(), device=dsts.device), lens)
        off = torch.cumsum(lens, 0) - lens
        pos = starts[seg] + torch.arange(int(lens.sum()), device=dsts.device) - off[seg]
        j = col[pos].long()
        nodes, inv = torch.unique(torch.cat([j, dsts]), return_inverse=True)
        return {"nodes": nodes.cpu(), "jl": inv[:j.numel()].cpu(), "il": inv[j.numel():].cpu(),
                "seg": seg.cpu(), "n": dsts.numel(), "rows": nodes.numel(), "dsts": dsts.cpu()}

    @staticmethod
    def run_from(x_host: torch.Tensor, idx: dict, weight: torch.Tensor, att_src: torch.Tensor,
                 att_dst: torch.Tensor, bias: Optional[torch.Tensor],
                 heads: int = 8) -> torch.Tensor:
        """``run`` with the row gather out of the full host x inside (the
        dataflow's index_select of the source rows, cache behaviour included)."""
        sub = dict(idx)
        sub["x"] = x_host.index_select(0, idx["nodes"]).float()
        return gatconv_forward_sampled.run(sub, weight, att_src, att_dst, bias, heads)

    @staticmethod
    def run(sub: dict, weight: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor,
            bias: Optional[torch.Tensor], heads: int = 8) -> torch.Tensor:
        H = heads
        C = weight.size(0) // H
        h = (sub["x"] @ weight.t()).view(-1, H, C)
        a_src = (h * att_src.reshape(1, H, C)).sum(-1)
        a_dst = (h * att_dst.reshape(1, H, C)).sum(-1)
        jl, il, seg, n = sub["jl"], sub["il"], sub["seg"], sub["n"]
        logit = F.leaky_relu(a_src[jl] + a_dst[il][seg], NEG_SLOPE)
        alpha = segment_softmax(logit, seg, n)
        agg = torch.zeros((n, H, C), dtype=h.dtype).index_add(0, seg,
                                                                alpha.unsqueeze(-1) * h[jl])
        out = agg.mean(dim=1)
        return out + bias if bias is not None else out


def gatconv_grads_chunked(x: torch.Tensor, rowptr: torch.Tensor, col: torch.Tensor,
                          weight: torch.Tensor, att_src: torch.Tensor, att_dst: torch.Tensor,
                          bias: torch.Tensor, grad_out: torch.Tensor, heads: int = 8,
                          chunk_edges: int = 2_000_000, dtype=torch.float32,
                          kinks_from: Optional[torch.Tensor] = None) -> dict:
    """Gradients of ``sum(out * grad_out)`` for the PyG-dataflow forward on a
    destination-sorted CSR (self loops in), with the backward that autograd
    takes through it (train.py:142) -- at sizes where the ``[E', H, C]``
    message tensor does not fit: h = x W^T is computed once for every node;
    destination chunks of <= ``chunk_edges`` messages then run the logits,
    segment softmax and aggregation under autograd with the gathered h rows as
    leaves, and their row gradients are summed into dh ``[N, H*C]``; finally
    grad_W = dh^T x and grad_x = dh W.  att_src / att_dst / bias gradients
    accumulate through autograd chunk by chunk.  Returns a dict of CPU tensors
    (x, weight, att_src, att_dst, bias) in ``dtype`` (float64: a reference
    whose own rounding is negligible next to the fp32 tolerance at N ~ 1e6+),
    plus ``dh`` = dL/dh [N, H*C].

    ``kinks_from`` ([N, 2H] logits table s | t of the implementation under
    test): the pre-activations s_j + t_i take those VALUES (the gradient path
    is unchanged, a straight-through substitution), so LeakyReLU's derivative
    -- 1 or the slope, a jump at 0 -- is decided on the same side as in the
    implementation.  At 10^7+ messages some s_j + t_i lie within fp32
    rounding of 0, where any two correct fp32 computations may pick
    different sides and the gradient legitimately differs by O(1)."""
    N, Fin = x.shape
    H = heads
    C = weight.size(0) // H
    x = x.to(dtype)
    W = weight.detach().to(dtype)
    with torch.no_grad():
        h_all = x @ W.t()                                   # [N, H*C]
    a_s = att_src.detach().reshape(1, H, C).to(dtype).clone().requires_grad_(True)
    a_d = att_dst.detach().reshape(1, H, C).to(dtype).clone().requires_grad_(True)
    b = bias.detach().to(dtype).clone().requires_grad_(True)
    dh = torch.zeros_like(h_all)
    rp = rowptr.long()
    col = col.long()
    start = 0
    while start < N:
        e0 = int(rp[start])
        k = int(torch.searchsorted(rp, torch.tensor([e0 + chunk_edges]), right=True).item()) - 1
        stop = min(N, max(start + 1, k))
        e1 = int(rp[stop])
        j = col[e0:e1]
        seg = torch.repeat_interleave(torch.arange(stop - start),
                                      (rp[start + 1:stop + 1] - rp[start:stop]))
        dsts = torch.arange(start, stop)
        rows, inv = torch.unique(torch.cat([j, dsts]), return_inverse=True)
        hr = h_all[rows].view(-1, H, C).clone().requires_grad_(True)
        jl, il = inv[:j.numel()], inv[j.numel():]
        a_src = (hr * a_s).sum(-1)
        a_dst = (hr * a_d).sum(-1)
        pre = a_src[jl] + a_dst[il][seg]
        if kinks_from is not None:
            kd = kinks_from[rows].to(dtype)
            pre_d = kd[jl, :H] + kd[il, H:][seg]
            pre = pre + (pre_d - pre).detach()
        logit = F.leaky_relu(pre, NEG_SLOPE)
        alpha = segment_softmax(logit, seg, stop - start)
        agg = torch.zeros((stop - start, H, C), dtype=hr.dtype).index_add(
            0, seg, alpha.unsqueeze(-1) * hr[jl])
        out = agg.mean(dim=1) + b
        (out * grad_out[start:stop].to(dtype)).sum().backward()
        dh.index_add_(0, rows, hr.grad.reshape(rows.numel(), H * C))
        start = stop
    return {"x": dh @ W, "weight": dh.t() @ x, "att_src": a_s.grad.reshape(att_src.shape),
            "att_dst": a_d.grad.reshape(att_dst.shape), "bias": b.grad, "dh": dh}


def glorot_(t: torch.Tensor, gen: Optional[torch.Generator] = None) -> torch.Tensor:
    """PyG ``inits.glorot``: U(-a, a), a = sqrt(6 / (fan_in + fan_out)) over the last two dims."""
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.copy_(torch.rand(t.shape, generator=gen, dtype=t.dtype) * 2 * a - a)
    return t


class GATConvRef(nn.Module):
    """PyG-2.x-compatible ``GATConv`` (``concat=False`` path) on the CPU.

    Parameter layout is PyG's for an int ``in_channels``: ``lin_src.weight``
    ``[H*C, F]`` with ``lin_dst`` the *same* module, ``att_src``/``att_dst``
    ``[1, H, C]``, ``bias`` ``[C]``.  Both state-dict keys ``lin_src.weight``
    and ``lin_dst.weight`` are emitted and accepted (the shipped checkpoints
    hold both, sharing storage).
    """

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = NEG_SLOPE, dropout: float = 0.0,
                 add_self_loops: bool = True, bias: bool = True, **kwargs):
        super().__init__()
        if concat:
            raise NotImplementedError("oracle restates the concat=False path used by the reference")
        if not add_self_loops:
            raise NotImplementedError("the reference always adds self loops")
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.lin_src = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.lin_dst = self.lin_src
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self, gen: Optional[torch.Generator] = None):
        glorot_(self.lin_src.weight, gen)
        glorot_(self.att_src, gen)
        glorot_(self.att_dst, gen)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor, edge_index: torch.Tensor) -> torch.Tensor:
        return gatconv_forward(x, edge_index, self.lin_src.weight, self.att_src, self.att_dst,
                               self.bias, heads=self.heads, negative_slope=self.negative_slope,
                               dropout=self.dropout, training=self.training)
