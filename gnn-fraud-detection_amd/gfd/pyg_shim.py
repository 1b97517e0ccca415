"""Make the reference's own model files run on gfd without editing them.

The reference imports ``from torch_geometric.nn import GATConv`` (gat.py:4,
tgn.py:4).  ``install()`` registers a minimal ``torch_geometric.nn`` module
whose ``GATConv`` is ``gfd.nn.GATConv``; importing ``src.models`` afterwards
gives the reference's GAT/TemporalGNN on the HIP path.  This is the one-line
swap a maintainer makes in the reference's training loop.
"""
from __future__ import annotations

import sys
import types

from .nn import GATConv


def install(force: bool = False) -> None:
    if "torch_geometric" in sys.modules and not force:
        mod = sys.modules.get("torch_geometric.nn")
        if mod is not None and getattr(mod, "GATConv", None) is GATConv:
            return
        if not force:
            raise RuntimeError("a real torch_geometric is already imported; pass force=True")
    tg = types.ModuleType("torch_geometric")
    tgnn = types.ModuleType("torch_geometric.nn")
    tgnn.GATConv = GATConv
    tg.nn = tgnn
    sys.modules["torch_geometric"] = tg
    sys.modules["torch_geometric.nn"] = tgnn
