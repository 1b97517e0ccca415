"""GPU neighbour sampling (replaces PyG NeighborLoader,
/root/reference/src/data/dataloader.py:42-66, num_neighbors [10, 10, 10],
batch_size 256).

CPU: Floyd's algorithm in the oracle draws uniform k-subsets (chi-square over
many seeds) and the restated sampler's invariants on a small CSR.
GPU: gfd_sample_neighbors bit-exact against oracle/sample_ref.py (same
counter-based draws) on an Elliptic-shaped graph with hubs; every sampled edge
exists; per-node counts are min(k, in-degree); the loader runs the
reference's training step on sampled batches."""
import numpy as np
import pytest
import torch

DEV = "cuda"


def _csr(N, ei):
    """gfd's CSR layout on the host: dst-sorted, stable, self loops dropped and
    one appended per node (the GATConv CSR the sampler walks)."""
    src, dst = ei
    keep = src != dst
    src, dst = src[keep], dst[keep]
    order = np.argsort(dst, kind="stable")
    rowptr = np.zeros(N + 1, np.int64)
    np.add.at(rowptr, dst + 1, 1)
    rowptr = np.cumsum(rowptr)
    col = []
    for i in range(N):
        col += src[order[rowptr[i]:rowptr[i + 1]]].tolist() + [i]
    rp = rowptr + np.arange(N + 1)
    return rp, np.array(col, np.int64)


def test_floyd_is_uniform():
    from oracle import floyd
    d, k, trials = 30, 7, 6000
    hist = np.zeros(d)
    for s in range(trials):
        p = floyd(d, k, seed=s, hop=0, node=5)
        assert len(set(p)) == k and all(0 <= t < d for t in p)
        hist[p] += 1
    exp = trials * k / d
    chi2 = ((hist - exp) ** 2 / exp).sum()
    assert chi2 < 70, chi2          # 29 dof: p ~ 1e-5 at 70


def test_sample_ref_invariants():
    from oracle import sample_ref
    rng = np.random.default_rng(0)
    N = 300
    ei = rng.integers(0, N, size=(2, 3000))
    rp, col = _csr(N, ei)
    seeds = rng.choice(N, 20, replace=False)
    n_id, level, edges, eptr = sample_ref(rp, col, seeds, [5, 3], seed=9)
    assert n_id[:20] == seeds.tolist() and len(set(n_id)) == len(n_id)
    for (s, d, e) in edges:
        assert col[e] == n_id[s] and rp[n_id[d]] <= e < rp[n_id[d] + 1] - 1
    for hop, k in enumerate([5, 3]):
        for f in range(level[hop], level[hop + 1]):
            deg = rp[n_id[f] + 1] - rp[n_id[f]] - 1
            got = sum(1 for (s, d, e) in edges[eptr[hop]:eptr[hop + 1]] if d == f)
            assert got == min(k, deg)


@pytest.mark.gpu
@pytest.mark.parametrize("fanouts", [[10, 10, 10], [25, 5]])
def test_sampler_matches_oracle(fanouts):
    from gfd import synth
    from gfd.sampler import NeighborSampler
    from oracle import sample_ref
    g = synth.elliptic_like(num_nodes=20000, num_edges=60000, num_steps=10, num_features=8, seed=4)
    ei = torch.from_numpy(g["edge_index"]).to(DEV)
    smp = NeighborSampler(ei, 20000, fanouts, seed=123)
    rp = smp.graph.rowptr.cpu().numpy()
    col = smp.graph.col.cpu().numpy()
    seeds = torch.randperm(20000, generator=torch.Generator().manual_seed(1))[:256]
    b = smp.sample(seeds)
    n_id, level, edges, eptr = sample_ref(rp, col, seeds.tolist(), fanouts, 123)
    assert b.n_id.cpu().tolist() == n_id
    assert b.level_ptr == level and b.edge_ptr == eptr
    e = np.array(edges, np.int64).T
    assert np.array_equal(b.edge_index.cpu().numpy(), e[:2])
    assert np.array_equal(b.edge_id.cpu().numpy(), e[2])
    assert (smp.local_of == -1).all()            # scratch map left clean
    b2 = smp.sample(seeds)                       # deterministic per seed
    assert torch.equal(b2.n_id, b.n_id) and torch.equal(b2.edge_index, b.edge_index)


@pytest.mark.gpu
def test_sampler_hub_uniformity():
    """A node with in-degree 200 sampled with k = 10 under 400 seeds: each
    in-neighbour is drawn with probability 10 / 200."""
    from gfd.sampler import NeighborSampler
    N = 1000
    src = torch.arange(1, 201)
    ei = torch.stack([src, torch.zeros(200, dtype=torch.long)]).to(DEV)
    smp = NeighborSampler(ei, N, [10], seed=0)
    hist = torch.zeros(N)
    for s in range(400):
        b = smp.sample(torch.tensor([0]), seed=s)
        assert b.edge_index.size(1) == 10
        picked = b.n_id[b.edge_index[0]].cpu()
        assert picked.unique().numel() == 10
        hist[picked] += 1
    h = hist[1:201].numpy()
    exp = 400 * 10 / 200
    chi2 = ((h - exp) ** 2 / exp).sum()
    assert chi2 < 280, chi2                       # 199 dof


@pytest.mark.gpu
def test_loader_training_step_on_sampled_batches():
    """The reference's mini-batch step (train.py:103-110) on gfd batches: GAT
    forward on the sampled subgraph, BCE on the seeds, backward."""
    from gfd import synth
    from gfd.models import GAT
    from gfd.sampler import NeighborLoader
    g = synth.elliptic_like(num_nodes=20000, num_edges=40000, num_steps=8, num_features=165, seed=2)
    x = torch.from_numpy(g["x"]).to(DEV)
    y = torch.from_numpy(g["y"]).to(DEV)
    ei = torch.from_numpy(g["edge_index"]).to(DEV)
    loader = NeighborLoader(x, ei, [10, 10, 10], batch_size=256, input_nodes=y != -1,
                            shuffle=True, y=y, seed=1)
    m = GAT(165, 64, 1, num_layers=3).to(DEV).train()
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], device=DEV))
    seen = 0
    for k, batch in enumerate(loader):
        out = m(batch.x, batch.edge_index)[:batch.batch_size].squeeze(1)
        loss = crit(out, batch.y[:batch.batch_size].float())
        loss.backward()
        assert torch.isfinite(loss)
        seen += batch.batch_size
        if k == 3:
            break
    assert seen == 4 * 256
    assert all(torch.isfinite(p.grad).all() for p in m.parameters() if p.grad is not None)


def test_batch_seeds_do_not_collide_across_fields():
    """(seed, epoch, batch) -> draw stream: tuples that overlapping bit fields
    would merge (batch 2^20 of epoch e vs batch 0 of e + 1; epochs >= 2^12 vs
    the user seed) get distinct streams."""
    from gfd.sampler import batch_seed
    assert batch_seed(0, 0, 2 ** 20) != batch_seed(0, 1, 0)
    assert batch_seed(0, 2 ** 12, 0) != batch_seed(1, 0, 0)
    seen = {batch_seed(s, e, b) for s in range(3) for e in range(20) for b in range(200)}
    assert len(seen) == 3 * 20 * 200
