"""Fused inference paths of the reference model bodies.

* ``gat_layer`` -- one layer of /root/reference/src/models/gat.py:79-91 (and
  tgn.py:93-105) in eval mode: GATConv -> BatchNorm1d(running stats) -> ReLU
  -> dropout (identity) -> residual, as ONE call of ``gfd_gat_fwd_ep``: the
  BatchNorm folds into a per-channel affine applied where the tile kernels
  store each output row, so the layer output is written once (the unfused
  path writes the GATConv output, then BN, ReLU and the residual add each
  read and write [N, 64] again).
* ``gru_head`` -- the TemporalGNN head (tgn.py:108-111): GRUCell(h, h0) +
  Linear in one kernel (``gfd_gru_head``); ``tgn_head_train`` -- the same
  head in training mode, forward and backward on the device
  (``gfd_gru_head_bwd`` + ``gfd_atb``).

* ``train_body`` -- the same layer body in training mode after the GATConv:
  residual + dropout(relu(BatchNorm1d(y))) with batch statistics, as one
  autograd Function over ``gfd_bn_relu_fwd`` / ``gfd_bn_relu_bwd`` (two
  passes over y each way instead of ATen's BN / relu / dropout / add chain
  and its saved intermediates; only y and two [64] vectors are kept).

``gat_layer`` and ``gru_head`` are inference-only: they refuse tensors that
require grad (gfd.models takes ``GATConv`` + ``train_body`` then).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _lib
from .graph import CSRGraph, _ws, get_graph
from .nn import SUPPORTED_CHANNELS, SUPPORTED_HEADS, _rows

H, C = SUPPORTED_HEADS, SUPPORTED_CHANNELS


def bn_affine(bn: Optional[torch.nn.BatchNorm1d], device) -> torch.Tensor:
    """[2C] (scale | shift) of an eval-mode BatchNorm1d: y = x * scale + shift
    with scale = gamma / sqrt(running_var + eps), shift = beta - mean * scale
    (identity when ``bn`` is None)."""
    if bn is None:
        return torch.cat([torch.ones(C, device=device), torch.zeros(C, device=device)])
    if not bn.track_running_stats or bn.running_var is None:
        raise NotImplementedError("fused BatchNorm needs running statistics (eval mode)")
    scale = torch.rsqrt(bn.running_var.float() + bn.eps)
    if bn.affine:
        scale = scale * bn.weight.float()
    shift = -bn.running_mean.float() * scale
    if bn.affine:
        shift = shift + bn.bias.float()
    return torch.cat([scale, shift]).contiguous()


def head_foldable(head, width: int, conv=None) -> bool:
    """The model head the store can fold (gfd_epilogue.head_*): Linear(64, 1)
    in fp32 after a layer whose input width takes the plan-scheduled kernels
    (F <= 168) and, when ``conv`` (the last GATConv) is given, whose attention
    slope those kernels take (leaky01: negative_slope in [0, 1]; others go to
    the head-less k_fused path, which cannot fold the head -- ADVICE r4)."""
    if conv is not None and not (0.0 <= float(conv.negative_slope) <= 1.0):
        return False
    return (head is not None and head.in_features == C and head.out_features == 1 and
            head.weight.dtype == torch.float32 and head.weight.is_cuda and width <= 168 and
            (head.bias is None or head.bias.dtype == torch.float32))


def check_params(conv, bn, device) -> None:
    """The checks GATConvFunction.forward makes on the layer's tensors, for the
    packed-weights inference paths (eval_conv, gat_layer): their pointers go
    to the kernels on x's stream, so a parameter left on the CPU, on another
    GPU or in another dtype must raise here, not fault or read garbage there
    (ADVICE r5)."""
    from .nn import _check_tensor
    _check_tensor("lin_src.weight", conv.lin_src.weight, device)
    _check_tensor("att_src", conv.att_src, device)
    _check_tensor("att_dst", conv.att_dst, device)
    if conv.bias is not None:
        _check_tensor("bias", conv.bias, device)
    if bn is not None:
        for n in ("running_mean", "running_var", "weight", "bias"):
            t = getattr(bn, n, None)
            if t is not None:
                _check_tensor(f"BatchNorm {n}", t, device)


def eval_weights(conv, bn, device) -> Tuple[torch.Tensor, torch.Tensor]:
    """(packed weights, BatchNorm scale | shift) of an inference layer, rebuilt
    only when a tensor they derive from changed: the cache on ``conv`` holds
    each source tensor, its version counter and storage address, so a replaced
    parameter (a new object), an in-place update (optimizer step,
    load_state_dict) or new storage (``.to(device)``) rebuilds it, while
    evaluation over many batches (evaluate.py:73-98) packs once."""
    srcs = [conv.lin_src.weight, conv.att_src, conv.att_dst]
    if bn is not None:
        srcs += [bn.running_mean, bn.running_var]
        if bn.affine:
            srcs += [bn.weight, bn.bias]
    # (object, version, storage address): a module moved to another device or
    # given new .data keeps its parameter objects but not their storage
    key = [(t, t._version, t.data_ptr()) for t in srcs] + [bn.eps if bn is not None else None,
                                                             bn, str(device)]
    c = conv.__dict__.get("_gfd_eval")
    if c is not None and len(c[0]) == len(key) and all(
            (a[0] is b[0] and a[1:] == b[1:]) if isinstance(a, tuple) else a is b or a == b
            for a, b in zip(c[0], key)):
        return c[1], c[2]
    W = conv.lin_src.weight.detach().contiguous()
    F = W.size(1)
    lib = _lib.load()
    packed = torch.empty(lib.gfd_gat_packed_size(F, H, C), dtype=torch.uint8, device=device)
    _lib.call("gfd_gat_pack_weights", W.data_ptr(),
              conv.att_src.detach().reshape(-1).contiguous().data_ptr(),
              conv.att_dst.detach().reshape(-1).contiguous().data_ptr(), F, H, C,
              packed.data_ptr(), _lib.stream_handle(device))
    ab = bn_affine(bn, device)
    conv.__dict__["_gfd_eval"] = (key, packed, ab)
    return packed, ab


def eval_conv(conv, x: torch.Tensor, edge_index) -> torch.Tensor:
    """``conv(x, edge_index)`` in inference (no autograd, no dropout) with the
    layer's packed weights from ``eval_weights``: the drop-in module's
    ``torch.no_grad()`` forward (gat.py:80 under evaluate.py:73-98)."""
    from .nn import _check_tensor
    dev = x.device
    _check_tensor("x", x, dev, (torch.float32, torch.bfloat16))
    graph = edge_index if isinstance(edge_index, CSRGraph) else get_graph(edge_index, x.size(0))
    if graph.num_nodes != x.size(0):
        raise ValueError(f"graph has {graph.num_nodes} nodes but x has {x.size(0)} rows")
    x = _rows(x)
    N, F = x.shape
    if F != conv.lin_src.weight.size(1):
        raise ValueError(f"x has {F} features, the layer expects {conv.lin_src.weight.size(1)}")
    check_params(conv, None, dev)
    packed, _ = eval_weights(conv, None, dev)
    bias = conv.bias.detach() if conv.bias is not None else None
    plan = graph.plan()
    lib = _lib.load()
    out = torch.empty((N, C), dtype=torch.float32, device=dev)
    ws = _ws(lib.gfd_gat_fwd_workspace_size(N, N, F, H, C, plan.num_hubs, plan.num_chunks), dev)
    _lib.call("gfd_gat_fwd_ep_packed", x.data_ptr(), _lib.x_dtype_code(x), N, F, x.stride(0),
              graph.rowptr.data_ptr(), graph.col.data_ptr(), packed.data_ptr(), _lib.ptr(bias),
              H, C, float(conv.negative_slope), 0.0, 0, plan.cstruct(), None, out.data_ptr(),
              None, None, ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
    return out


def gat_layer(conv, bn, h: torch.Tensor, edge_index, relu: bool = True,
              residual: bool = False, head=None) -> torch.Tensor:
    """One eval-mode layer body: residual(h) + relu(bn(conv(h, edge_index))).
    ``head`` (Linear(64, 1), see head_foldable): the model head folded into
    the store (gat.py:94) -- returns head(body) [N, 1] and the [N, 64] body
    is never written."""
    if torch.is_grad_enabled() and (h.requires_grad or conv.lin_src.weight.requires_grad):
        raise RuntimeError("gfd.fused.gat_layer is inference-only (use torch.no_grad())")
    dev = h.device
    graph = edge_index if isinstance(edge_index, CSRGraph) else get_graph(edge_index, h.size(0))
    x = _rows(h)
    N, F = x.shape
    bias = conv.bias.detach() if conv.bias is not None else None
    check_params(conv, bn, dev)
    packed, ab = eval_weights(conv, bn, dev)
    res = None
    if residual:
        if F != C:
            raise ValueError("residual needs the layer input width to equal 64")
        # the epilogue adds fp32 rows (gfd_epilogue.residual is float*)
        res = x if x.dtype == torch.float32 else x.float()
    hout = hw = None
    if head is not None:
        if not head_foldable(head, F, conv):
            raise ValueError("gat_layer head: Linear(64, 1) fp32 on the device after a layer the "
                             "plan-scheduled kernels take (head_foldable)")
        hw = head.weight.detach().reshape(-1).contiguous()
        hout = torch.empty((N, 1), dtype=torch.float32, device=dev)
    ep = _lib.GfdEpilogue(ab.data_ptr(), 1 if relu else 0, _lib.ptr(res),
                          res.stride(0) if res is not None else 0, _lib.ptr(hw),
                          _lib.ptr(head.bias.detach() if head is not None and
                                   head.bias is not None else None), _lib.ptr(hout))
    plan = graph.plan()
    lib = _lib.load()
    out = torch.empty((N, C), dtype=torch.float32, device=dev) if hout is None else None
    ws = _ws(lib.gfd_gat_fwd_workspace_size(N, N, F, H, C, plan.num_hubs, plan.num_chunks), dev)
    _lib.call("gfd_gat_fwd_ep_packed", x.data_ptr(), _lib.x_dtype_code(x), N, F, x.stride(0),
              graph.rowptr.data_ptr(), graph.col.data_ptr(), packed.data_ptr(), _lib.ptr(bias),
              H, C, float(conv.negative_slope), 0.0, 0, plan.cstruct(), _lib.ct.byref(ep),
              _lib.ptr(out), None, None, ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
    return out if hout is None else hout


def gru_head(gru: torch.nn.GRUCell, lin: torch.nn.Linear, h: torch.Tensor,
             h0: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """(lin(GRUCell(h, h0)), GRUCell(h, h0)) in one kernel (h0 None = zeros)."""
    if torch.is_grad_enabled() and (h.requires_grad or gru.weight_ih.requires_grad):
        raise RuntimeError("gfd.fused.gru_head is inference-only (use torch.no_grad())")
    if gru.hidden_size != C or gru.input_size != C:
        raise NotImplementedError("gfd gru_head: GRUCell(64, 64)")
    dev = h.device
    x = h.float() if h.dtype != torch.float32 else h      # the kernel reads fp32 rows
    x = x if x.stride(1) == 1 and x.stride(0) % 4 == 0 else x.contiguous()
    if h0 is not None:
        h0 = h0.float() if h0.dtype != torch.float32 else h0
        h0 = h0 if h0.stride(1) == 1 and h0.stride(0) % 4 == 0 else h0.contiguous()
    N = x.size(0)
    O = lin.out_features
    h_new = torch.empty((N, C), dtype=torch.float32, device=dev)
    out = torch.empty((N, O), dtype=torch.float32, device=dev)
    w_ih, w_hh = gru.weight_ih.detach().contiguous(), gru.weight_hh.detach().contiguous()
    b_ih = gru.bias_ih.detach() if gru.bias else None
    b_hh = gru.bias_hh.detach() if gru.bias else None
    w_o = lin.weight.detach().contiguous()
    b_o = lin.bias.detach() if lin.bias is not None else None
    _lib.call("gfd_gru_head", x.data_ptr(), N, C, x.stride(0), w_ih.data_ptr(), _lib.ptr(b_ih),
              w_hh.data_ptr(), _lib.ptr(b_hh), _lib.ptr(h0), h0.stride(0) if h0 is not None else 0,
              w_o.data_ptr(), _lib.ptr(b_o), O, h_new.data_ptr(), out.data_ptr(),
              _lib.stream_handle(dev))
    return out, h_new


class _GRUHeadTrain(torch.autograd.Function):
    """(out, h_new) = (Linear(GRUCell(h, h0)), GRUCell(h, h0)) with both
    directions on the device: forward = gfd_gru_head (the inference kernel:
    gates on fp32 MFMA, nothing but h / h0 / h_new kept), backward =
    gfd_gru_head_bwd (gates recomputed, gate gradients, grad_h / grad_h0) +
    gfd_atb for the six weight / bias gradients (deterministic sums)."""

    @staticmethod
    def forward(ctx, h, h0, w_ih, b_ih, w_hh, b_hh, w_o, b_o):
        dev = h.device
        N = h.size(0)
        O = w_o.size(0)
        h_new = torch.empty((N, C), dtype=torch.float32, device=dev)
        out = torch.empty((N, O), dtype=torch.float32, device=dev)
        _lib.call("gfd_gru_head", h.data_ptr(), N, C, h.stride(0), w_ih.data_ptr(), _lib.ptr(b_ih),
                  w_hh.data_ptr(), _lib.ptr(b_hh), _lib.ptr(h0),
                  h0.stride(0) if h0 is not None else 0, w_o.data_ptr(), _lib.ptr(b_o), O,
                  h_new.data_ptr(), out.data_ptr(), _lib.stream_handle(dev))
        ctx.save_for_backward(h, h0, w_ih, b_ih, w_hh, b_hh, w_o, b_o, h_new)
        return out, h_new

    @staticmethod
    def backward(ctx, g_out, g_hnew):
        h, h0, w_ih, b_ih, w_hh, b_hh, w_o, b_o, h_new = ctx.saved_tensors
        dev = h.device
        N, O = h.size(0), w_o.size(0)
        lib = _lib.load()
        stream = _lib.stream_handle(dev)
        g_out = (g_out if g_out is not None else torch.zeros((N, O), device=dev)).float().contiguous()
        g_hnew = g_hnew.float().contiguous() if g_hnew is not None else None
        grad_h = torch.empty((N, C), dtype=torch.float32, device=dev)
        grad_h0 = torch.empty((N, C), dtype=torch.float32, device=dev) if h0 is not None else None
        gi = torch.empty((N, 3 * C), dtype=torch.float32, device=dev)
        gh = torch.empty_like(gi)
        _lib.call("gfd_gru_head_bwd", h.data_ptr(), N, C, h.stride(0), w_ih.data_ptr(),
                  _lib.ptr(b_ih), w_hh.data_ptr(), _lib.ptr(b_hh), _lib.ptr(h0),
                  h0.stride(0) if h0 is not None else 0, w_o.data_ptr(), O, g_out.data_ptr(),
                  _lib.ptr(g_hnew), grad_h.data_ptr(), _lib.ptr(grad_h0), gi.data_ptr(),
                  gh.data_ptr(), stream)
        ws = _ws(lib.gfd_atb_workspace_size(N, 3 * C), dev)

        def atb(A, m, B):
            wgt = torch.empty((m, C), dtype=torch.float32, device=dev)
            col = torch.empty((m,), dtype=torch.float32, device=dev)
            _lib.call("gfd_atb", A.data_ptr(), A.stride(0), m, _lib.ptr(B),
                      B.stride(0) if B is not None else C, N, wgt.data_ptr(), col.data_ptr(),
                      ws.data_ptr(), ws.numel(), stream)
            return wgt, col

        g_wih, g_bih = atb(gi, 3 * C, h)
        if h0 is not None:
            g_whh, g_bhh = atb(gh, 3 * C, h0)
        else:                                   # h0 = 0: no W_hh product, only b_hh
            g_whh = torch.zeros_like(w_hh)
            g_bhh = atb(gh, 3 * C, h)[1]
        g_wo, g_bo = atb(g_out, O, h_new)
        return (grad_h, grad_h0, g_wih, g_bih if b_ih is not None else None, g_whh,
                g_bhh if b_hh is not None else None, g_wo, g_bo if b_o is not None else None)


def _aligned_rows(t: torch.Tensor) -> torch.Tensor:
    """t itself when its rows are unit-stride, 16-B aligned and at a 16-B
    multiple pitch (what gfd_gru_head / _bwd read as vectors); otherwise a
    fresh contiguous copy -- also for a contiguous view at a misaligned offset,
    which .contiguous() would return unchanged."""
    if t.stride(1) == 1 and t.stride(0) % 4 == 0 and t.data_ptr() % 16 == 0:
        return t
    return t.clone(memory_format=torch.contiguous_format)


def tgn_head_train(gru: torch.nn.GRUCell, lin: torch.nn.Linear, h: torch.Tensor,
                   h0: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """Training form of ``gru_head``: (lin(GRUCell(h, h0)), GRUCell(h, h0)) as
    one autograd Function over gfd_gru_head / gfd_gru_head_bwd / gfd_atb
    (tgn.py:108-111 under loss.backward(), train.py:142)."""
    if gru.hidden_size != C or gru.input_size != C or not gru.bias:
        raise NotImplementedError("gfd tgn_head_train: GRUCell(64, 64) with biases")
    x = _aligned_rows(h if h.dtype == torch.float32 else h.float())
    if h0 is not None:
        h0 = _aligned_rows(h0.float() if h0.dtype != torch.float32 else h0)
    b_o = lin.bias
    return _GRUHeadTrain.apply(x, h0, gru.weight_ih.contiguous(), gru.bias_ih,
                               gru.weight_hh.contiguous(), gru.bias_hh, lin.weight.contiguous(),
                               b_o)


class _BNReluDropout(torch.autograd.Function):
    """out = res + dropout(relu(bn_train(y))); see include/gfd.h gfd_bn_relu_fwd."""

    @staticmethod
    def forward(ctx, y, res, gamma, beta, bn, relu, p, seed):
        dev = y.device
        N = y.size(0)
        lib = _lib.load()
        ws = _ws(lib.gfd_bn_workspace_size(), dev)
        out = torch.empty_like(y)
        mean = torch.empty(C, dtype=torch.float32, device=dev)
        invstd = torch.empty_like(mean)
        momentum = bn.momentum
        if bn.track_running_stats and bn.num_batches_tracked is not None:
            bn.num_batches_tracked.add_(1)
            if momentum is None:  # cumulative moving average (torch BatchNorm semantics)
                momentum = 1.0 / float(bn.num_batches_tracked.item())
        rm = bn.running_mean if bn.track_running_stats else None
        rv = bn.running_var if bn.track_running_stats else None
        _lib.call("gfd_bn_relu_fwd", y.data_ptr(), _lib.ptr(res), N, C, _lib.ptr(gamma),
                  _lib.ptr(beta), float(bn.eps), float(momentum or 0.0), _lib.ptr(rm),
                  _lib.ptr(rv), 1 if relu else 0, float(p), seed, out.data_ptr(),
                  mean.data_ptr(), invstd.data_ptr(), ws.data_ptr(), ws.numel(),
                  _lib.stream_handle(dev))
        ctx.save_for_backward(y, gamma, beta, mean, invstd)
        ctx.relu, ctx.p, ctx.seed, ctx.has_res = relu, p, seed, res is not None
        return out

    @staticmethod
    def backward(ctx, gout):
        y, gamma, beta, mean, invstd = ctx.saved_tensors
        gout = gout.contiguous()
        dev = y.device
        lib = _lib.load()
        ws = _ws(lib.gfd_bn_workspace_size(), dev)
        gy = torch.empty_like(y)
        gg = torch.empty(C, dtype=torch.float32, device=dev)
        gb = torch.empty_like(gg)
        _lib.call("gfd_bn_relu_bwd", y.data_ptr(), gout.data_ptr(), y.size(0), C,
                  gamma.data_ptr(), beta.data_ptr(), mean.data_ptr(), invstd.data_ptr(),
                  1 if ctx.relu else 0, float(ctx.p), ctx.seed, gy.data_ptr(), gg.data_ptr(),
                  gb.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle(dev))
        return (gy, gout if ctx.has_res else None, gg, gb, None, None, None, None)


def train_supported(bn, y: torch.Tensor) -> bool:
    """Whether ``train_body`` takes this layer: an affine training-mode
    BatchNorm1d(64) over fp32 [N, 64] rows on the GPU."""
    return (bn is not None and bn.training and bn.affine and y.is_cuda
            and y.dtype == torch.float32 and y.dim() == 2 and y.size(1) == C and y.size(0) > 1
            and bn.weight.dtype == torch.float32)


def train_body(y: torch.Tensor, bn: torch.nn.BatchNorm1d, h: Optional[torch.Tensor],
               relu: bool = True, p: float = 0.0) -> torch.Tensor:
    """(h +) dropout(relu(bn(y)), p) in training mode (gat.py:82-91).  The
    dropout mask is drawn from a seed taken from torch's CPU generator, so
    ``torch.manual_seed`` makes it reproducible (it is not torch's own mask)."""
    y = y.contiguous()
    res = None
    if h is not None:
        res = h if (h.dtype == torch.float32 and h.is_contiguous()) else h.float().contiguous()
    seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if p > 0 else 0
    return _BNReluDropout.apply(y, res, bn.weight, bn.bias, bn, relu, p, seed)
