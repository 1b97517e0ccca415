"""Destination-sharded multi-GPU execution.

One process per GPU (``torch.distributed``, backend "nccl" = RCCL on ROCm).
Ownership is by DESTINATION node: every in-edge of a destination lives on its
owner, so the segment softmax and the aggregation are rank-local and only
source-side data crosses GPUs.  Shards are contiguous destination ranges
balanced by message count (prefix sum over in-degree).

Layer 0 keeps ``x`` halo-resident (every rank holds the rows its in-edges
reference; for a power-law graph that is nearly all of x).  The per-node
attention logits are then computed for the rank's own destination block and
exchanged with one RCCL all-gather of ``[N, 2H]`` fp32 (the "halo" of the
north star: 64 B per node instead of the 664 B feature row), after which the
fused aggregate-project kernel runs on the local shard with no further
communication.  Hidden layers all-gather the previous layer's ``[N, 64]``
output instead.
"""
from __future__ import annotations

from typing import List, Tuple

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
