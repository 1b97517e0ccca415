"""Per-time-step snapshot extraction (config C3; the reference's
create_temporal_subgraph, /root/reference/src/data/dataset.py:198-240, per step
of create_temporal_dataloaders, dataloader.py:99-135).

CPU: the vectorised oracle against the reference's own per-edge loop (restated
in oracle/temporal_ref.py) on small graphs, including a known answer.
GPU: gfd.temporal (gfd_temporal_snapshots, every step in one pass) bit-exact
against the oracle for every step, on an Elliptic-shaped graph with injected
cross-step edges, out-of-range time steps and an empty step; and the TGN
snapshot forward against per-step oracle forwards on such a graph."""
import numpy as np
import pytest
import torch

from _util import assert_close

DEV = "cuda"


def _graph(N=3000, E=6000, steps=7, cross=400, seed=0):
    from gfd import synth
    g = synth.elliptic_like(num_nodes=N, num_edges=E, num_steps=steps, num_features=16, seed=seed)
    rng = np.random.default_rng(seed)
    ei = g["edge_index"]
    extra = rng.integers(0, N, size=(2, cross))                    # mostly cross-step edges
    ei = np.concatenate([ei, extra], axis=1)
    ei = ei[:, rng.permutation(ei.shape[1])]
    return g, ei.astype(np.int64)


def test_oracle_known_answer():
    from oracle import temporal_subgraph_ref
    ts = np.array([1, 2, 1, 2, 1])
    ei = np.array([[0, 1, 2, 4, 3, 0],
                   [2, 3, 4, 0, 0, 4]])
    nodes, local, kept = temporal_subgraph_ref(ts, ei, 1)
    assert nodes.tolist() == [0, 2, 4]
    assert kept.tolist() == [0, 2, 3, 5]
    assert local.tolist() == [[0, 1, 2, 0], [1, 2, 0, 2]]
    nodes, local, kept = temporal_subgraph_ref(ts, ei, 2)
    assert nodes.tolist() == [1, 3] and kept.tolist() == [1] and local.tolist() == [[0], [1]]


def test_oracle_matches_reference_loop():
    from oracle import temporal_subgraph_loop, temporal_subgraph_ref
    g, ei = _graph(N=400, E=900, steps=5, cross=60)
    for t in range(0, 7):
        a = temporal_subgraph_ref(g["time_step"], ei, t)
        b = temporal_subgraph_loop(g["time_step"].tolist(), ei.tolist(), t)
        for u, v in zip(a, b):
            assert np.array_equal(u, v)


@pytest.mark.gpu
def test_snapshots_match_oracle_every_step():
    from gfd.temporal import temporal_snapshots
    from oracle import temporal_subgraph_ref
    g, ei = _graph()
    ts = g["time_step"].copy()
    ts[::97] = 100                                  # outside the extracted range
    ts[ts == 3] = 4                                 # step 3 is empty
    snap = temporal_snapshots(torch.from_numpy(ts).to(DEV), torch.from_numpy(ei).to(DEV),
                              ts.size, t_first=1, num_steps=7)
    x = torch.arange(ts.size, device=DEV).float()
    total = 0
    for t in range(1, 8):
        nodes, local, kept = temporal_subgraph_ref(ts, ei, t)
        sub = snap.subgraph(t, x=x)
        assert sub["node_indices"].cpu().numpy().tolist() == nodes.tolist()
        assert np.array_equal(sub["edge_index"].cpu().numpy(), local)
        assert np.array_equal(sub["x"].cpu().numpy(), nodes.astype(np.float32))
        e0, e1 = snap.edge_ptr[t - 1], snap.edge_ptr[t]
        assert np.array_equal(snap.edge_index_intra[:, e0:e1].cpu().numpy(), ei[:, kept])
        total += kept.size
    assert snap.edge_ptr[-1] == total
    assert snap.step_ptr[-1] == int(((ts >= 1) & (ts <= 7)).sum())
    pos = snap.node_pos.cpu().numpy()
    assert np.array_equal(snap.node_perm.cpu().numpy()[pos], np.arange(ts.size))


@pytest.mark.gpu
def test_snapshot_forward_matches_per_step_oracle():
    """TemporalGNN.forward_snapshots on a graph WITH cross-step edges equals
    the reference's per-step forwards on create_temporal_subgraph outputs."""
    from gfd.models import TemporalGNN
    from oracle import TemporalGNNRef, temporal_subgraph_ref
    from gfd import synth
    torch.manual_seed(0)
    g = synth.elliptic_like(num_nodes=2500, num_edges=5000, num_steps=6, num_features=40, seed=3)
    rng = np.random.default_rng(3)
    ei = np.concatenate([g["edge_index"], rng.integers(0, 2500, size=(2, 500))], axis=1)
    ref = TemporalGNNRef(40, 64, 1, num_layers=3).eval()
    m = TemporalGNN(40, 64, 1, num_layers=3).to(DEV).eval()
    m.load_state_dict(ref.state_dict(), strict=True)
    x = torch.from_numpy(g["x"])
    with torch.no_grad():
        out, hid = m.forward_snapshots(x.to(DEV), torch.from_numpy(ei).to(DEV),
                                       torch.from_numpy(g["time_step"]).to(DEV))
        want = torch.zeros(2500, 1)
        want_h = torch.zeros(2500, 64)
        for t in range(1, 7):
            nodes, local, _ = temporal_subgraph_ref(g["time_step"], ei, t)
            o, h = ref(x[nodes], torch.from_numpy(local))
            want[nodes], want_h[nodes] = o, h
    assert_close(out, want, what="TGN snapshot out")
    assert_close(hid, want_h, what="TGN snapshot hidden")
