"""CPU restatement of the reference's per-time-step subgraph extraction --
TEST INFRASTRUCTURE ONLY (the checker for gfd.temporal / gfd_temporal_snapshots).

Follows ``create_temporal_subgraph`` (/root/reference/src/data/dataset.py:198-240):
  * nodes: ``mask = time_steps == t``, ``node_indices = nonzero(mask)`` -- the
    step's nodes in ascending id order (:210-211);
  * ``idx_mapping = {old id: position}`` (:214);
  * edges: kept when both endpoints are in the mapping, in their original order
    (:217-222), then relabelled through the mapping (:225-229);
  * x, y and time_steps restricted to ``node_indices`` (:232-237).
The reference's membership test ``src in idx_mapping`` (:220) looks up a 0-d
tensor among int keys; tensors hash by identity, so as written it keeps no edge.
This restatement follows the function's documented intent ("only nodes and
edges from the specified time step"); parity for the edge filter is therefore
"unpinned" against the reference's literal behaviour.
"""
from __future__ import annotations

import numpy as np


def temporal_subgraph_ref(time_steps: np.ndarray, edge_index: np.ndarray, t: int):
    """(node_indices [n_t], edge_index_local [2, e_t], kept_edge_ids [e_t])."""
    time_steps = np.asarray(time_steps)
    edge_index = np.asarray(edge_index)
    node_indices = np.nonzero(time_steps == t)[0]                     # dataset.py:210-211
    mapping = np.full(time_steps.shape[0], -1, dtype=np.int64)        # dataset.py:214
    mapping[node_indices] = np.arange(node_indices.size)
    src, dst = edge_index[0], edge_index[1]
    keep = (mapping[src] >= 0) & (mapping[dst] >= 0)                  # dataset.py:217-220
    kept = np.nonzero(keep)[0]
    local = np.stack([mapping[src[kept]], mapping[dst[kept]]])        # dataset.py:225-229
    return node_indices, local.astype(np.int64), kept


def temporal_subgraph_loop(time_steps, edge_index, t: int):
    """The same with the reference's per-edge Python loop and dict (small inputs)."""
    node_indices = [i for i, s in enumerate(time_steps) if s == t]
    idx_mapping = {int(idx): i for i, idx in enumerate(node_indices)}
    kept, local = [], []
    for e in range(len(edge_index[0])):
        s, d = int(edge_index[0][e]), int(edge_index[1][e])
        if s in idx_mapping and d in idx_mapping:
            kept.append(e)
            local.append((idx_mapping[s], idx_mapping[d]))
    loc = np.array(local, dtype=np.int64).T.reshape(2, -1)
    return np.array(node_indices, dtype=np.int64), loc, np.array(kept, dtype=np.int64)
