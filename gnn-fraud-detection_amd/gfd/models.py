"""Reference model families on the HIP GATConv.

``GAT`` mirrors /root/reference/src/models/gat.py (ctor :14-58, forward
:60-96, predict :98-122) and ``TemporalGNN`` mirrors
/root/reference/src/models/tgn.py (ctor :18-63, forward :67-113) -- same
constructor arguments, same submodule names (so ``results/gat_model.pt`` and
``results/tgn_model.pt`` load with ``strict=True``), same outputs.  The only
difference is the GATConv underneath: ``gfd.nn.GATConv`` (libgfd.so).

The per-layer epilogue is the reference's: GATConv -> BatchNorm1d -> ReLU ->
dropout -> residual when widths match (gat.py:79-91).  In inference (eval mode
under no_grad) each layer is one fused call (BN folded into the GATConv store
epilogue, ``gfd.fused.gat_layer``) and the TemporalGNN head is one kernel
(``gfd.fused.gru_head``); in training the body after each GATConv (batch-
statistics BN, ReLU, dropout, residual) is one autograd Function over two
kernels each way (``gfd.fused.train_body``), and the TemporalGNN head is one
too (``gfd.fused.tgn_head_train``: GRUCell + Linear forward and backward).

``forward_snapshots`` is config C3: the TGN forward over per-time-step
snapshots (h0 = 0 per step, tgn.py:88-89).  Elliptic edges never cross time
steps, so the 49 snapshot forwards are one block-diagonal launch over the
step-sorted graph; the result equals the per-step forwards exactly in eval
mode (checked against the reference in tests/golden).
"""
from __future__ import annotations

from typing import Optional, Tuple

import torch
import torch.nn as nn
import torch.nn.functional as F

from .nn import GATConv


class _GATStack(nn.Module):
    """The GATConv/BN/ReLU/dropout/residual stack shared by both families."""

    def __init__(self, in_channels: int, hidden_channels: int, out_channels: int,
                 num_layers: int = 2, dropout: float = 0.2, residual: bool = True,
                 use_batch_norm: bool = True):
        super().__init__()
        self.in_channels, self.hidden_channels = in_channels, hidden_channels
        self.out_channels, self.num_layers = out_channels, num_layers
        self.dropout, self.residual, self.use_batch_norm = dropout, residual, use_batch_norm
        # layer 0 takes in_channels, every later layer hidden_channels (gat.py:39-56)
        widths = [in_channels] + [hidden_channels] * max(num_layers - 1, 0)
        self.gat_layers = nn.ModuleList(
            GATConv(w, hidden_channels, heads=8, concat=False, dropout=dropout) for w in widths)
        self.batch_norms = (nn.ModuleList(nn.BatchNorm1d(hidden_channels) for _ in widths)
                            if use_batch_norm else None)

    def _fused(self) -> bool:
        """Inference (eval mode, no autograd): each layer body runs as one
        GATConv launch chain with BN/ReLU/residual in the store epilogue."""
        return not self.training and not torch.is_grad_enabled()

    def encode(self, x: torch.Tensor, edge_index, head=None) -> torch.Tensor:
        """The layer stack; in inference, ``head`` (fused.head_foldable) is
        folded into the last layer's store and its [N, 1] output returned."""
        h = x
        if self._fused():
            from . import fused
            last = len(self.gat_layers) - 1
            for layer, conv in enumerate(self.gat_layers):
                bn = self.batch_norms[layer] if self.batch_norms is not None else None
                h = fused.gat_layer(conv, bn, h, edge_index, relu=True,
                                    residual=self.residual and h.size(-1) == self.hidden_channels,
                                    head=head if layer == last else None)
            return h
        for layer, conv in enumerate(self.gat_layers):
            y = conv(h, edge_index)
            bn = self.batch_norms[layer] if self.batch_norms is not None else None
            if self.training and bn is not None:
                from . import fused
                if fused.train_supported(bn, y):
                    res = h if (self.residual and h.size(-1) == y.size(-1)) else None
                    h = fused.train_body(y, bn, res, relu=True, p=self.dropout)
                    continue
            if self.batch_norms is not None:
                y = self.batch_norms[layer](y)
            y = F.dropout(F.relu(y), p=self.dropout, training=self.training)
            h = h + y if (self.residual and h.size(-1) == y.size(-1)) else y
        return h


def _head(lin: nn.Linear, h: torch.Tensor) -> torch.Tensor:
    """``lin(h)``.  For the reference's single-logit head (Linear(64, 1),
    gat.py:58, tgn.py:63) as a row-wise dot product: ATen maps the [N, 64] x
    [64, 1] product and its weight gradient (a K = N reduction) onto GEMM
    tiles that took 0.45 ms of a 6.7-ms Elliptic-size train step; the
    elementwise form is a multiply and two reductions."""
    if lin.out_features == 1 and h.dim() == 2 and h.is_cuda:
        y = (h * lin.weight).sum(-1, keepdim=True)
        return y + lin.bias if lin.bias is not None else y
    return lin(h)


class GAT(_GATStack):
    """Drop-in for ``src.models.gat.GAT``."""

    def __init__(self, in_channels: int, hidden_channels: int, out_channels: int,
                 num_layers: int = 2, dropout: float = 0.2, residual: bool = True,
                 use_batch_norm: bool = True):
        super().__init__(in_channels, hidden_channels, out_channels, num_layers, dropout,
                         residual, use_batch_norm)
        self.out = nn.Linear(hidden_channels, out_channels)

    def forward(self, x, edge_index, batch: Optional[torch.Tensor] = None) -> torch.Tensor:
        if self._fused() and x.is_cuda and self.gat_layers:
            from .fused import head_foldable
            width = self.gat_layers[-1].in_channels
            if head_foldable(self.out, width, self.gat_layers[-1]):
                # inference: Linear(64, 1) folded into the last layer's store
                # (gat.py:94): the [N, 64] body is never written or re-read
                return self.encode(x, edge_index, head=self.out)
        return _head(self.out, self.encode(x, edge_index))

    def predict(self, x, edge_index, batch=None, apply_sigmoid: bool = True) -> torch.Tensor:
        out = self.forward(x, edge_index, batch)
        return torch.sigmoid(out) if apply_sigmoid else out


class TemporalGNN(_GATStack):
    """Drop-in for ``src.models.tgn.TemporalGNN``: GAT stack -> GRUCell -> Linear."""

    def __init__(self, in_channels: int, hidden_channels: int, out_channels: int,
                 num_layers: int = 2, dropout: float = 0.2, residual: bool = True,
                 use_batch_norm: bool = True):
        super().__init__(in_channels, hidden_channels, out_channels, num_layers, dropout,
                         residual, use_batch_norm)
        self.gru = nn.GRUCell(hidden_channels, hidden_channels)
        self.out = nn.Linear(hidden_channels, out_channels)

    def forward(self, x, edge_index, batch: Optional[torch.Tensor] = None,
                hidden_state: Optional[torch.Tensor] = None) -> Tuple[torch.Tensor, torch.Tensor]:
        h = self.encode(x, edge_index)
        if self._fused():
            from . import fused
            return fused.gru_head(self.gru, self.out, h, hidden_state)
        if h.is_cuda and self._device_head_ok():
            # training / autograd: GRUCell + Linear forward and backward on the
            # device (gfd.fused.tgn_head_train); h0 = None is the reference's zeros
            from . import fused
            return fused.tgn_head_train(self.gru, self.out, h, hidden_state)
        if hidden_state is None:
            hidden_state = x.new_zeros((x.size(0), self.hidden_channels))
        new_hidden = self.gru(h, hidden_state)
        return _head(self.out, new_hidden), new_hidden

    def _device_head_ok(self) -> bool:
        """The head kernels' set: GRUCell(64, 64) with biases, Linear(64, <= 64),
        fp32 parameters (anything else -- e.g. a .double() model -- takes the
        torch GRUCell + Linear path instead of being read as fp32)."""
        g, o = self.gru, self.out
        params = list(g.parameters()) + list(o.parameters())
        return (g.bias and g.input_size == g.hidden_size == 64 and o.in_features == 64 and
                o.out_features <= 64 and all(p.dtype == torch.float32 for p in params))

    def predict(self, x, edge_index, batch=None, hidden_state=None,
                apply_sigmoid: bool = True) -> torch.Tensor:
        out, _ = self.forward(x, edge_index, batch, hidden_state)
        return torch.sigmoid(out) if apply_sigmoid else out

    def forward_snapshots(self, x: torch.Tensor, edge_index: torch.Tensor,
                          time_step: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
        """Config C3: the forward of every time-step snapshot (the reference's
        create_temporal_subgraph per step, dataset.py:198-240, h0 = 0 per step,
        tgn.py:88-89) in one launch chain: the snapshots are extracted on the
        device (gfd.temporal) and run side by side as one graph that keeps only
        intra-step edges, so every destination sees exactly its own step.
        Exact per-snapshot semantics in eval mode (train-mode BatchNorm would
        take batch statistics over all steps instead of one)."""
        from .temporal import cached_snapshots
        snap = cached_snapshots(time_step, edge_index, x.size(0))
        return self.forward(x, snap.edge_index_intra)
