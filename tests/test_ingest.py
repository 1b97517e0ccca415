"""Graph ingest (gfd.ingest; EllipticBitcoinDataset.process,
/root/reference/src/data/dataset.py:75-129) against the restatement in
oracle/ingest_ref.py on synthetic CSVs in the Elliptic layout (the real CSVs are
not in the reference): a header-less features file (pandas turns the first
transaction into the header), a repeated transaction id,
edges and class rows naming unknown ids, 'unknown' labels."""
import os

import numpy as np
import pytest
import torch

DEV = "cuda"


def _write_csvs(d, N=500, E=1500, F=12, seed=0):
    rng = np.random.default_rng(seed)
    ids = rng.choice(10 ** 9, N, replace=False).astype(np.int64) + 10 ** 8
    ids[17] = ids[3]                                   # a repeated id
    ts = rng.integers(1, 50, N)
    x = rng.standard_normal((N, F)).round(5)
    with open(os.path.join(d, "elliptic_txs_features.csv"), "w") as f:
        for i in range(N):                             # no header row (as in Elliptic)
            f.write(",".join([str(ids[i]), str(ts[i])] + [f"{v:.5f}" for v in x[i]]) + "\n")
    src = rng.choice(ids, E)
    dst = rng.choice(ids, E)
    src[::50] = 7                                      # unknown ids
    dst[::70] = ids[0]                                 # the id that became the header
    with open(os.path.join(d, "elliptic_txs_edgelist.csv"), "w") as f:
        f.write("txId1,txId2\n")
        for a, b in zip(src, dst):
            f.write(f"{a},{b}\n")
    lab = rng.choice(["1", "2", "unknown"], N)
    cid = ids.copy()
    cid[5] = 11                                        # unknown id
    with open(os.path.join(d, "elliptic_txs_classes.csv"), "w") as f:
        f.write("txId,class\n")
        for a, b in zip(cid, lab):
            f.write(f"{a},{b}\n")
        f.write(f"{ids[9]},1\n")                       # a later row relabels node 9
    return ids


def test_oracle_known_structure(tmp_path):
    from oracle import process_ref
    ids = _write_csvs(str(tmp_path))
    r = process_ref(str(tmp_path))
    assert r["x"].shape == (499, 12)                   # the first row became the header
    assert r["edge_index"].shape[0] == 2
    assert (r["edge_index"] >= 0).all() and (r["edge_index"] < 499).all()
    assert set(np.unique(r["y"]).tolist()) <= {-1, 0, 1}


def test_binary_roundtrip_cpu(tmp_path):
    from gfd.ingest import load_graph, save_graph
    x = torch.randn(100, 7)
    ei = torch.randint(0, 100, (2, 300))
    save_graph(str(tmp_path / "g"), x=x, edge_index=ei)
    back = load_graph(str(tmp_path / "g"), device="cpu")
    assert torch.equal(back["x"], x) and torch.equal(back["edge_index"], ei)


@pytest.mark.gpu
def test_ingest_matches_reference_process(tmp_path):
    from gfd.ingest import ingest_elliptic
    from oracle import process_ref
    _write_csvs(str(tmp_path), N=3000, E=9000, F=20, seed=1)
    ref = process_ref(str(tmp_path))
    got = ingest_elliptic(str(tmp_path), DEV)
    assert np.array_equal(got["edge_index"].cpu().numpy(), ref["edge_index"])
    assert np.array_equal(got["y"].cpu().numpy(), ref["y"])
    assert np.array_equal(got["time_steps"].cpu().numpy(), ref["time_steps"])
    assert np.array_equal(got["x"].cpu().numpy(), ref["x"])


@pytest.mark.gpu
def test_binary_load_streams_to_device_and_runs_model(tmp_path):
    from gfd import synth
    from gfd.ingest import load_graph, save_graph
    from gfd.models import GAT
    g = synth.elliptic_like(num_nodes=50000, num_edges=60000, num_steps=10, num_features=165, seed=0)
    save_graph(str(tmp_path / "g"), x=torch.from_numpy(g["x"]),
               edge_index=torch.from_numpy(g["edge_index"]), y=torch.from_numpy(g["y"]))
    d = load_graph(str(tmp_path / "g"), DEV)
    assert d["x"].is_cuda and torch.equal(d["x"].cpu(), torch.from_numpy(g["x"]))
    assert torch.equal(d["edge_index"].cpu(), torch.from_numpy(g["edge_index"]))
    m = GAT(165, 64, 1, num_layers=3).to(DEV).eval()
    with torch.no_grad():
        out = m(d["x"], d["edge_index"])
    assert out.shape == (50000, 1) and torch.isfinite(out).all()
