"""CPU restatement of the reference model wiring -- TEST INFRASTRUCTURE ONLY.

Restates ``GAT`` (/root/reference/src/models/gat.py:10-96) and
``TemporalGNN`` (/root/reference/src/models/tgn.py:13-113) around the oracle
``GATConvRef``.  Pinned against ``tests/golden/*.npz``, which were produced by
the reference's own modules (see tests/golden/make_golden.py).  Used only by
tests to check the product models on random graphs no fixture covers.
"""
from __future__ import annotations

from typing import Optional

import torch
import torch.nn as nn
import torch.nn.functional as F

from .gatconv_ref import GATConvRef


class GATRef(nn.Module):
    """gat.py:14-58 (ctor) and :60-96 (forward)."""

    def __init__(self, in_channels, hidden_channels, out_channels, num_layers=2, dropout=0.2,
                 residual=True, use_batch_norm=True):
        super().__init__()
        self.hidden_channels, self.dropout = hidden_channels, dropout
        self.residual, self.use_batch_norm = residual, use_batch_norm
        self.gat_layers = nn.ModuleList()
        self.batch_norms = nn.ModuleList() if use_batch_norm else None
        widths = [in_channels] + [hidden_channels] * (num_layers - 1)  # gat.py:39,45,51
        for w in widths:
            self.gat_layers.append(GATConvRef(w, hidden_channels, heads=8, concat=False, dropout=dropout))
            if use_batch_norm:
                self.batch_norms.append(nn.BatchNorm1d(hidden_channels))
        self.out = nn.Linear(hidden_channels, out_channels)

    def body(self, x, edge_index):
        h = x
        for i, gat in enumerate(self.gat_layers):            # gat.py:79-91
            h_new = gat(h, edge_index)
            if self.use_batch_norm:
                h_new = self.batch_norms[i](h_new)
            h_new = F.relu(h_new)
            h_new = F.dropout(h_new, p=self.dropout, training=self.training)
            h = h + h_new if (self.residual and h.size(-1) == h_new.size(-1)) else h_new
        return h

    def forward(self, x, edge_index, batch=None):
        return self.out(self.body(x, edge_index))             # gat.py:94


class TemporalGNNRef(GATRef):
    """tgn.py:67-113: the GAT stack, then ``GRUCell(h, h0)`` (h0 = zeros unless
    given, tgn.py:88-89), then ``Linear`` on the new hidden state."""

    def __init__(self, in_channels, hidden_channels, out_channels, num_layers=2, dropout=0.2,
                 residual=True, use_batch_norm=True):
        super().__init__(in_channels, hidden_channels, out_channels, num_layers, dropout,
                         residual, use_batch_norm)
        self.gru = nn.GRUCell(hidden_channels, hidden_channels)   # tgn.py:60

    def forward(self, x, edge_index, batch=None, hidden_state: Optional[torch.Tensor] = None):
        if hidden_state is None:
            hidden_state = torch.zeros(x.size(0), self.hidden_channels, dtype=x.dtype)
        h = self.body(x, edge_index)
        hidden_state = self.gru(h, hidden_state)                  # tgn.py:108
        return self.out(hidden_state), hidden_state               # tgn.py:111-113
