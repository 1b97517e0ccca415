"""Synthetic graph generators for the SURVEY.md §8d configurations.

The Elliptic CSVs are absent (``/root/reference/elliptic_bitcoin_dataset/data.txt``
holds only a download link), so every workload is synthetic, shaped after the
reference's own statistics:

* ``elliptic_like`` -- C1/C2/C3: 49 time steps, edges only inside a step
  (consistent with ``create_temporal_subgraph``, dataset.py:198-240), src/dst
  skewed inside a step, no self loops; the reference's COO layout
  (``edge_index[0]`` = source, ``[1]`` = destination, dataset.py:104).
  Defaults are the Elliptic shape (processed_data/dataset_stats.json:2-5).
* ``power_law`` -- C4/C5: Chung-Lu with in/out weights
  ``w_i ∝ (i + 10) ** (-1 / (gamma - 1))`` and randomly permuted ids.

All generators are deterministic functions of ``seed`` (numpy PCG64 on the
host; ``power_law_device`` uses a torch generator on the target device and is
deterministic per device type).
"""
from __future__ import annotations

import numpy as np

ELLIPTIC_NODES = 203_769
ELLIPTIC_EDGES = 234_355
ELLIPTIC_STEPS = 49
GENERATOR_VERSION = 1


def _step_sizes(num_nodes: int, num_steps: int, rng: np.random.Generator) -> np.ndarray:
    # per-step node counts between ~1.1k and ~7.9k at full scale (time_step_distribution.png)
    prof = 1100.0 + 6800.0 * rng.random(num_steps)
    sizes = np.floor(prof / prof.sum() * num_nodes).astype(np.int64)
    sizes = np.maximum(sizes, 2)
    sizes[np.argmax(sizes)] += num_nodes - sizes.sum()
    assert sizes.sum() == num_nodes and (sizes >= 2).all()
    return sizes


def elliptic_like(num_nodes: int = ELLIPTIC_NODES, num_edges: int = ELLIPTIC_EDGES,
                  num_steps: int = ELLIPTIC_STEPS, num_features: int = 166, seed: int = 0,
                  labelled_frac: float = 0.23, illicit_frac: float = 0.098):
    """Return a dict with ``x [N,F] f32``, ``edge_index [2,E] i64``,
    ``time_step [N] i64`` (1-based), ``y [N] i64`` (-1 unknown, 0 licit, 1 illicit).

    Nodes are numbered step by step (block-diagonal by time step)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    sizes = _step_sizes(num_nodes, num_steps, rng)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    e_per = np.floor(sizes / sizes.sum() * num_edges).astype(np.int64)
    e_per[np.argmax(e_per)] += num_edges - e_per.sum()
    src_l, dst_l = [], []
    for s in range(num_steps):
        n, m = int(sizes[s]), int(e_per[s])
        perm = rng.permutation(n)
        got_s, got_d = [], []
        need = m
        while need > 0:
            a = perm[np.minimum((n * rng.random(need) ** 3).astype(np.int64), n - 1)]
            b = perm[np.minimum((n * rng.random(need) ** 2).astype(np.int64), n - 1)]
            keep = a != b
            got_s.append(a[keep]); got_d.append(b[keep])
            need -= int(keep.sum())
        src_l.append(np.concatenate(got_s)[:m] + starts[s])
        dst_l.append(np.concatenate(got_d)[:m] + starts[s])
    edge_index = np.stack([np.concatenate(src_l), np.concatenate(dst_l)]).astype(np.int64)
    x = rng.standard_normal((num_nodes, num_features), dtype=np.float32)
    time_step = np.repeat(np.arange(1, num_steps + 1), sizes).astype(np.int64)
    y = np.full(num_nodes, -1, dtype=np.int64)
    lab = rng.random(num_nodes) < labelled_frac
    y[lab] = (rng.random(int(lab.sum())) < illicit_frac).astype(np.int64)
    return {"x": x, "edge_index": edge_index, "time_step": time_step, "y": y,
            "step_sizes": sizes}


def chung_lu_weights(num_nodes: int, gamma: float = 2.1) -> np.ndarray:
    return (np.arange(num_nodes, dtype=np.float64) + 10.0) ** (-1.0 / (gamma - 1.0))


def power_law(num_nodes: int, num_edges: int, gamma: float = 2.1, seed: int = 1) -> np.ndarray:
    """Host Chung-Lu generator (small/medium sizes). Returns ``edge_index [2,E] i64``."""
    rng = np.random.Generator(np.random.PCG64(seed))
    cdf = np.cumsum(chung_lu_weights(num_nodes, gamma))
    cdf /= cdf[-1]
    perm = rng.permutation(num_nodes)
    src = perm[np.minimum(np.searchsorted(cdf, rng.random(num_edges), side="right"), num_nodes - 1)]
    dst = perm[np.minimum(np.searchsorted(cdf, rng.random(num_edges), side="right"), num_nodes - 1)]
    return np.stack([src, dst]).astype(np.int64)


def power_law_device(num_nodes: int, num_edges: int, gamma: float = 2.1, seed: int = 1,
                     device="cuda", chunk: int = 1 << 24):
    """Device-side Chung-Lu generator for C4/C5 sizes (10M/50M, 50M/500M).
    Returns an int64 ``[2, E]`` tensor on ``device``."""
    import torch
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    w = (torch.arange(num_nodes, dtype=torch.float64, device=device) + 10.0) ** (-1.0 / (gamma - 1.0))
    cdf = torch.cumsum(w, 0)
    cdf /= cdf[-1].clone()
    del w
    perm = torch.randperm(num_nodes, generator=g, device=device)
    out = torch.empty((2, num_edges), dtype=torch.int64, device=device)
    for row in range(2):
        for s in range(0, num_edges, chunk):
            n = min(chunk, num_edges - s)
            u = torch.rand(n, generator=g, dtype=torch.float64, device=device)
            idx = torch.searchsorted(cdf, u, right=True).clamp_(max=num_nodes - 1)
            out[row, s:s + n] = perm[idx]
    return out
