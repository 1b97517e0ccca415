"""Drop-in ``GATConv`` on the HIP library.

Replaces ``from torch_geometric.nn import GATConv`` at
/root/reference/src/models/gat.py:4 and tgn.py:4.  Same constructor subset as
the reference uses (``GATConv(in, out, heads=8, concat=False, dropout=p)``,
gat.py:39,45,51; tgn.py:43,49,55), same call (``conv(x, edge_index)``,
gat.py:80, tgn.py:94), same parameters and state-dict keys as PyG 2.x for an
int ``in_channels``: ``lin_src.weight [H*C, F]`` with ``lin_dst`` the same
module (both keys saved and accepted), ``att_src``/``att_dst [1, H, C]``,
``bias [C]`` -- the shipped checkpoints load with ``strict=True``.

Forward and backward both run in libgfd.so (``gfd_gat_fwd`` /
``gfd_gat_bwd``); there is no CPU or eager-PyTorch fallback.
"""
from __future__ import annotations

import math
import os
import weakref
from collections import OrderedDict
from typing import Optional

import torch
import torch.nn as nn

from . import _lib
from .graph import CSRGraph, _ws, get_graph

SUPPORTED_HEADS = 8
SUPPORTED_CHANNELS = 64


def _check_tensor(name: str, t: torch.Tensor, device, dtypes=(torch.float32,)):
    if not t.is_cuda:
        raise RuntimeError(f"gfd GATConv: {name} must be on a HIP device (got {t.device})")
    if t.device != device:
        raise RuntimeError(f"gfd GATConv: {name} is on {t.device}, expected {device}")
    if t.dtype not in dtypes:
        raise TypeError(f"gfd GATConv: {name} must be {' or '.join(map(str, dtypes))} "
                        f"(got {t.dtype})")


def _rows(x: torch.Tensor) -> torch.Tensor:
    """x with unit feature stride (any row pitch is passed through as is)."""
    return x if x.stride(1) == 1 and x.stride(0) >= x.size(1) else x.contiguous()


class GATConvFunction(torch.autograd.Function):
    """autograd.Function around gfd_gat_fwd / gfd_gat_bwd."""

    @staticmethod
    def forward(ctx, x, weight, att_src, att_dst, bias, graph: CSRGraph, negative_slope: float,
                dropout_p: float, seed: int, grad_mode: bool = True):
        dev = x.device
        _check_tensor("x", x, dev, (torch.float32, torch.bfloat16))
        for n, t in (("weight", weight), ("att_src", att_src), ("att_dst", att_dst)):
            _check_tensor(n, t, dev)
        if bias is not None:
            _check_tensor("bias", bias, dev)
        x = _rows(x)
        weight = weight.contiguous()
        att_src = att_src.contiguous()
        att_dst = att_dst.contiguous()
        N, F = x.shape
        HC = weight.size(0)
        H, C = SUPPORTED_HEADS, HC // SUPPORTED_HEADS
        plan = graph.plan()
        # the softmax statistics only for a backward: not under no_grad (the
        # module's parameters require grad even in inference; grad_mode is the
        # caller's torch.is_grad_enabled(), which is off inside forward)
        need_stats = grad_mode and any(ctx.needs_input_grad[:5])
        out = torch.empty((N, C), dtype=torch.float32, device=dev)
        st = torch.empty((N, 2 * H), dtype=torch.float32, device=dev)
        stats = torch.empty((N, 2 * H), dtype=torch.float32, device=dev) if need_stats else None
        lib = _lib.load()
        ws = _ws(lib.gfd_gat_fwd_workspace_size(N, N, F, H, C, plan.num_hubs, plan.num_chunks), dev)
        _lib.call("gfd_gat_fwd", x.data_ptr(), _lib.x_dtype_code(x), N, F, x.stride(0),
                  graph.rowptr.data_ptr(),
                  graph.col.data_ptr(), weight.data_ptr(), att_src.data_ptr(), att_dst.data_ptr(),
                  _lib.ptr(bias), H, C, float(negative_slope), float(dropout_p),
                  int(seed) & (2 ** 64 - 1), plan.cstruct(), out.data_ptr(), st.data_ptr(),
                  _lib.ptr(stats), ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
        if need_stats:
            ctx.save_for_backward(x, weight, att_src, att_dst, st, stats)
            ctx.graph = graph
            ctx.meta = (float(negative_slope), float(dropout_p), int(seed), bias is not None)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        x, weight, att_src, att_dst, st, stats = ctx.saved_tensors
        graph: CSRGraph = ctx.graph
        slope, dp, seed, has_bias = ctx.meta
        dev = x.device
        g = grad_out.contiguous().to(torch.float32)
        if g.data_ptr() % 16:  # the C-ABI reads grad_out rows as 16-B vectors
            g = g.clone()
        N, F = x.shape
        H, C = SUPPORTED_HEADS, weight.size(0) // SUPPORTED_HEADS
        csc = graph.csc()
        gx = torch.empty((N, F), dtype=torch.float32, device=dev) if ctx.needs_input_grad[0] else None
        gw = torch.empty_like(weight)
        gas = torch.empty_like(att_src)
        gad = torch.empty_like(att_dst)
        gb = torch.empty((C,), dtype=torch.float32, device=dev) if has_bias else None
        lib = _lib.load()
        plan, splan = graph.plan(), csc.plan
        ws = _ws(lib.gfd_gat_bwd_workspace_size(N, graph.num_messages, F, H, C, plan.num_hubs,
                                                plan.num_chunks, splan.num_chunks), dev)
        cm = x_colmax(x)
        _lib.call("gfd_gat_bwd_mode", x.data_ptr(), _lib.x_dtype_code(x), N, F, x.stride(0),
                  graph.rowptr.data_ptr(), graph.col.data_ptr(), plan.cstruct(),
                  csc.colptr.data_ptr(), csc.dst.data_ptr(), csc.eid.data_ptr(), splan.cstruct(),
                  graph.num_messages, weight.data_ptr(), att_src.data_ptr(),
                  att_dst.data_ptr(), H, C, slope, dp, seed & (2 ** 64 - 1), st.data_ptr(),
                  stats.data_ptr(), g.data_ptr(), _lib.ptr(gx), gw.data_ptr(), gas.data_ptr(),
                  gad.data_ptr(), _lib.ptr(gb), cm.data_ptr(), bwd_mode(), ws.data_ptr(),
                  ws.numel(), _lib.stream_handle(dev))
        if gx is not None and x.dtype != torch.float32:
            gx = gx.to(x.dtype)
        return gx, gw, gas, gad, gb, None, None, None, None, None


def bwd_mode() -> int:
    """The backward dataflow gfd_gat_bwd_mode is asked for: GFD_BWD_DH (0, the
    default) or, opt-in for A/B runs and tests, the fused source pass
    (environment GFD_BWD_FUSED=1: 8-wave blocks, =2: 16-wave).  Read here, per
    call, and passed explicitly: the C library itself reads no environment."""
    v = os.environ.get("GFD_BWD_FUSED", "0")
    return {"1": 1, "2": 2}.get(v, 0)


# Per-column maxima of |x| -- the scales of the backward's grad_W GEMM -- kept
# per version of the x tensor: the first layer's input is the same features
# tensor every training step (train.py:115-143), so gfd_x_colmax runs once for
# it.  Keyed on the tensor object (a weak reference: a new tensor at a recycled
# address is a different object) and its version counter (in-place updates).
_COLMAX: "OrderedDict[int, tuple]" = OrderedDict()
_COLMAX_ENTRIES = 8


def x_colmax(x: torch.Tensor) -> torch.Tensor:
    """uint32 [F] max |x[:, f]| as float bits (gfd_x_colmax), cached per x version."""
    ent = _COLMAX.get(id(x))
    if ent is not None:
        ref, ver, ptr, cm = ent
        if ref() is x and ver == x._version and ptr == x.data_ptr():
            _COLMAX.move_to_end(id(x))
            return cm
    cm = torch.empty(x.size(1), dtype=torch.int32, device=x.device)
    _lib.call("gfd_x_colmax", x.data_ptr(), _lib.x_dtype_code(x), x.size(0), x.size(1),
              x.stride(0), cm.data_ptr(), _lib.stream_handle(x.device))
    _COLMAX[id(x)] = (weakref.ref(x), x._version, x.data_ptr(), cm)
    while len(_COLMAX) > _COLMAX_ENTRIES:
        _COLMAX.popitem(last=False)
    return cm


def gat_conv(x: torch.Tensor, edge_index_or_graph, weight: torch.Tensor, att_src: torch.Tensor,
             att_dst: torch.Tensor, bias: Optional[torch.Tensor], negative_slope: float = 0.2,
             dropout: float = 0.0, training: bool = False) -> torch.Tensor:
    """Functional GATConv (heads=8, C=64, concat=False, self loops added)."""
    graph = edge_index_or_graph
    if not isinstance(graph, CSRGraph):
        graph = get_graph(edge_index_or_graph, x.size(0))
    if graph.num_nodes != x.size(0):
        raise ValueError(f"graph has {graph.num_nodes} nodes but x has {x.size(0)} rows")
    dp = float(dropout) if training else 0.0
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if dp > 0 else 0
    return GATConvFunction.apply(x, weight, att_src.reshape(-1), att_dst.reshape(-1), bias,
                                 graph, negative_slope, dp, seed, torch.is_grad_enabled())


def _glorot(t: torch.Tensor):
    a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
    with torch.no_grad():
        t.uniform_(-a, a)


class GATConv(nn.Module):
    """PyG-compatible ``GATConv`` for the reference's configuration.

    Supported: ``heads=8``, ``out_channels=64``, ``concat=False``,
    ``add_self_loops=True``, any ``in_channels <= 256``, optional bias; x in
    float32 or bfloat16 (config C5: converted exactly on load, fp32 arithmetic).
    Anything else raises ``NotImplementedError`` rather than computing
    something different from PyG.
    """

    def __init__(self, in_channels: int, out_channels: int, heads: int = 1, concat: bool = True,
                 negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 edge_dim: Optional[int] = None, fill_value="mean", bias: bool = True, **kwargs):
        super().__init__()
        if heads != SUPPORTED_HEADS or out_channels != SUPPORTED_CHANNELS or concat:
            raise NotImplementedError(
                "gfd GATConv implements the reference's configuration: heads=8, out_channels=64, "
                f"concat=False (got heads={heads}, out_channels={out_channels}, concat={concat})")
        if not add_self_loops or edge_dim is not None:
            raise NotImplementedError("gfd GATConv: add_self_loops=True and no edge features only")
        if not isinstance(in_channels, int) or not 1 <= in_channels <= 256:
            raise NotImplementedError("gfd GATConv: int in_channels in [1, 256]")
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.concat, self.negative_slope, self.dropout = concat, negative_slope, dropout
        self.add_self_loops = add_self_loops
        self.lin_src = nn.Linear(in_channels, heads * out_channels, bias=False)
        self.lin_dst = self.lin_src          # PyG aliases them for int in_channels
        self.att_src = nn.Parameter(torch.empty(1, heads, out_channels))
        self.att_dst = nn.Parameter(torch.empty(1, heads, out_channels))
        self.bias = nn.Parameter(torch.empty(out_channels)) if bias else None
        self.reset_parameters()

    def reset_parameters(self):
        _glorot(self.lin_src.weight)
        _glorot(self.att_src)
        _glorot(self.att_dst)
        if self.bias is not None:
            nn.init.zeros_(self.bias)

    def forward(self, x: torch.Tensor, edge_index, size=None, return_attention_weights=None):
        if return_attention_weights:
            raise NotImplementedError("gfd GATConv: return_attention_weights is not supported")
        if not torch.is_grad_enabled() and not (self.training and self.dropout > 0) and x.is_cuda:
            # inference: the packed weights are cached while the parameters do
            # not change (gfd.fused.eval_weights)
            from .fused import eval_conv
            return eval_conv(self, x, edge_index)
        return gat_conv(x, edge_index, self.lin_src.weight, self.att_src, self.att_dst, self.bias,
                        self.negative_slope, self.dropout, self.training)

    def extra_repr(self) -> str:
        return (f"{self.in_channels}, {self.out_channels}, heads={self.heads}, concat=False, "
                f"dropout={self.dropout}")
