"""GPU neighbour sampling: the reference's mini-batch mode.

Replaces ``torch_geometric.loader.NeighborLoader(data, num_neighbors=[10, 10,
10], batch_size=256, input_nodes=mask, shuffle=...)``
(/root/reference/src/data/dataloader.py:42-66; batch size config.py:41) with
``gfd_sample_neighbors`` on the device: every hop of a batch is sampled,
deduplicated and relabelled on the GPU; the graph never leaves HBM.

Each batch is a ``SampledBatch`` shaped like NeighborLoader's output:
``n_id`` (global node ids, the seeds first), ``edge_index`` ([2, E_b], local
ids, row 0 = source, row 1 = destination), ``batch_size`` (the seeds), plus
``x`` / ``y`` gathered from the full tensors when given, and the per-hop
boundaries.  The reference's training step on a batch (train.py:103-110) runs
unchanged on it; the loss is taken on the seeds (``[:batch_size]``) as PyG's
documentation prescribes (the reference takes it on every labelled sampled
node).

Sampling is uniform without replacement per node and hop (PyG's default),
deterministic per (seed, epoch, batch).  PyG's random stream itself cannot be
reproduced; the oracle (oracle/sample_ref.py) restates this algorithm with the
same counter-based draws and the tests compare bit-exactly, plus uniformity.
"""
from __future__ import annotations

import ctypes as ct
from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from . import _lib
from .graph import CSRGraph, _ws, get_graph, no_content_cache

_M64 = 2 ** 64 - 1


def _splitmix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


def batch_seed(seed: int, epoch: int, batch: int) -> int:
    """Per-batch sampling seed: the (seed, epoch, batch) tuple hashed field by
    field (splitmix64 chained), so no two tuples share a draw stream the way
    overlapping bit fields would (batch 2^20 of epoch e vs batch 0 of e + 1)."""
    h = _splitmix64(int(seed) & _M64)
    h = _splitmix64(h ^ (int(epoch) & _M64))
    return _splitmix64(h ^ (int(batch) & _M64))


@dataclass
class SampledBatch:
    n_id: torch.Tensor         # int64 [n]: global ids, seeds first
    edge_index: torch.Tensor   # int64 [2, e]: local ids (source, destination)
    edge_id: torch.Tensor      # int64 [e]: position of the edge in the CSR
    batch_size: int
    level_ptr: List[int]       # node offsets per hop (level 0 = seeds)
    edge_ptr: List[int]        # edge offsets per hop
    x: Optional[torch.Tensor] = None
    y: Optional[torch.Tensor] = None


class NeighborSampler:
    """Samples batches from a graph resident on the device."""

    def __init__(self, edge_index_or_graph, num_nodes: int, num_neighbors: Sequence[int],
                 seed: int = 0):
        g = edge_index_or_graph
        self.graph: CSRGraph = g if isinstance(g, CSRGraph) else get_graph(g, num_nodes)
        self.fanouts = (ct.c_int32 * len(num_neighbors))(*[int(k) for k in num_neighbors])
        self.hops = len(num_neighbors)
        self.seed = int(seed)
        dev = self.graph.device
        self.local_of = torch.full((self.graph.num_nodes,), -1, dtype=torch.int32, device=dev)
        self._ws = {}

    def _bounds(self, ns: int):
        lib = _lib.load()
        mn, me = _lib.c_i64(0), _lib.c_i64(0)
        _lib.call("gfd_sample_bounds", self.graph.num_nodes, ns, self.fanouts, self.hops,
                  ct.byref(mn), ct.byref(me))
        if ns not in self._ws:
            self._ws[ns] = _ws(lib.gfd_sample_workspace_size(self.graph.num_nodes, ns,
                                                             self.fanouts, self.hops),
                               self.graph.device)
        return mn.value, me.value, self._ws[ns]

    def sample(self, seeds: torch.Tensor, seed: Optional[int] = None,
               _unique: bool = False) -> SampledBatch:
        """``_unique``: the caller guarantees distinct seeds (NeighborLoader's
        batches are slices of a permutation of input nodes it checked once), so
        the per-batch sort + host sync of the duplicate check is skipped."""
        g = self.graph
        dev = g.device
        seeds = seeds.to(device=dev, dtype=torch.int64).contiguous()
        ns = seeds.numel()
        if ns == 0:
            raise ValueError("empty seed batch")
        if not _unique and torch.unique(seeds).numel() != ns:
            # the relabelling keeps one local id per node: a repeated seed
            # would silently lose its copy
            raise ValueError("seed batch holds duplicate node ids")
        mn, me, ws = self._bounds(ns)
        n_id = torch.empty(mn, dtype=torch.int64, device=dev)
        level_ptr = torch.empty(self.hops + 2, dtype=torch.int64, device=dev)
        esrc = torch.empty(max(me, 1), dtype=torch.int64, device=dev)
        edst = torch.empty(max(me, 1), dtype=torch.int64, device=dev)
        eid = torch.empty(max(me, 1), dtype=torch.int64, device=dev)
        edge_ptr = torch.empty(self.hops + 1, dtype=torch.int64, device=dev)
        st = _lib.load().gfd_sample_neighbors(
            g.rowptr.data_ptr(), g.col.data_ptr(), g.num_nodes, seeds.data_ptr(), ns,
            self.fanouts, self.hops, (self.seed if seed is None else int(seed)) & (2 ** 64 - 1),
            self.local_of.data_ptr(), n_id.data_ptr(), level_ptr.data_ptr(), esrc.data_ptr(),
            edst.data_ptr(), eid.data_ptr(), edge_ptr.data_ptr(), ws.data_ptr(), ws.numel(),
            _lib.stream_handle(dev))
        if st == 2:
            raise IndexError(f"a seed is outside [0, {g.num_nodes})")
        if st != 0:
            raise _lib.GfdError("gfd_sample_neighbors", st)
        lp, ep = level_ptr.tolist(), edge_ptr.tolist()
        n, e = lp[-1], ep[-1]
        ei = no_content_cache(torch.stack([esrc[:e], edst[:e]]))   # single-use subgraph
        return SampledBatch(n_id[:n], ei, eid[:e], ns, lp, ep)


class NeighborLoader:
    """Iterates sampled batches like PyG's NeighborLoader (dataloader.py:42-66):
    ``input_nodes`` (bool mask or index tensor), ``batch_size`` seeds per
    batch, ``shuffle`` (a new permutation per epoch), ``x`` / ``y`` gathered
    for the batch's nodes."""

    def __init__(self, x: torch.Tensor, edge_index, num_neighbors: Sequence[int],
                 batch_size: int, input_nodes: Optional[torch.Tensor] = None,
                 shuffle: bool = False, y: Optional[torch.Tensor] = None, seed: int = 0):
        self.x, self.y = x, y
        N = x.size(0)
        self.sampler = NeighborSampler(edge_index, N, num_neighbors, seed)
        dev = self.sampler.graph.device
        if input_nodes is None:
            idx = torch.arange(N, device=dev)
        elif input_nodes.dtype == torch.bool:
            idx = input_nodes.to(dev).nonzero().view(-1)
        else:
            idx = input_nodes.to(dev).long()
            if torch.unique(idx).numel() != idx.numel():
                raise ValueError("input_nodes holds duplicate node ids")
        self.input_nodes, self.batch_size, self.shuffle = idx, int(batch_size), shuffle
        self.seed, self.epoch = int(seed), 0

    def __len__(self):
        return (self.input_nodes.numel() + self.batch_size - 1) // self.batch_size

    def __iter__(self):
        idx = self.input_nodes
        if self.shuffle:
            gen = torch.Generator(device=idx.device)
            gen.manual_seed(self.seed * 1000003 + self.epoch)
            idx = idx[torch.randperm(idx.numel(), generator=gen, device=idx.device)]
        for b in range(len(self)):
            seeds = idx[b * self.batch_size:(b + 1) * self.batch_size]
            batch = self.sampler.sample(seeds, seed=batch_seed(self.seed, self.epoch, b),
                                        _unique=True)
            batch.x = self.x[batch.n_id]
            if self.y is not None:
                batch.y = self.y[batch.n_id]
            yield batch
        self.epoch += 1
