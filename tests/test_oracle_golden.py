"""CPU: the oracle (PyG-dataflow restatement) against the golden vectors that
the REFERENCE's own model code produced (tests/golden/make_golden.py).

This pins the oracle's model wiring (GAT/TGN layer order, BN/ReLU/residual,
GRU, head) and weights handling to the reference; the GATConv arithmetic is
PyG's published algorithm (parity unpinned vs real PyG, which is absent)."""
import numpy as np
import pytest
import torch

from _util import assert_close, assert_close_scaled, state_dict_from
from oracle import GATRef, TemporalGNNRef, gatconv_forward, remove_then_add_self_loops

torch.set_num_threads(4)


def _ref_model(cls, arr, prefix, dropout=0.2):
    m = cls(165, 64, 1, num_layers=3, dropout=dropout)
    m.load_state_dict(state_dict_from(arr, prefix), strict=True)
    return m


def test_checkpoint_shapes(golden):
    arr = golden("elliptic_small.npz")
    assert arr["gat.gat_layers.0.lin_src.weight"].shape == (512, 165)
    assert arr["gat.gat_layers.1.lin_src.weight"].shape == (512, 64)
    assert arr["tgn.gru.weight_ih"].shape == (192, 64)
    assert int(arr["gat.batch_norms.0.num_batches_tracked"]) == 100


def test_oracle_gat_matches_reference(golden):
    arr = golden("elliptic_small.npz")
    m = _ref_model(GATRef, arr, "gat.").eval()
    x, ei = torch.from_numpy(arr["x"]), torch.from_numpy(arr["edge_index"])
    with torch.no_grad():
        logits = m(x, ei)
    assert_close(logits, arr["gat_logits"], atol=1e-6, rtol=1e-6, what="oracle GAT logits")


def test_oracle_tgn_matches_reference(golden):
    arr = golden("elliptic_small.npz")
    m = _ref_model(TemporalGNNRef, arr, "tgn.").eval()
    x, ei = torch.from_numpy(arr["x"]), torch.from_numpy(arr["edge_index"])
    with torch.no_grad():
        out, hid = m(x, ei)
    assert_close(out, arr["tgn_out"], atol=1e-6, rtol=1e-6, what="oracle TGN out")
    assert_close(hid, arr["tgn_hidden"], atol=1e-6, rtol=1e-6, what="oracle TGN hidden")
    # block-diagonal time steps: full-graph forward == per-step snapshot forwards (eval)
    assert_close(out, arr["tgn_out_snapshots"], atol=1e-5, rtol=1e-5, what="snapshots")


def test_oracle_train_grads_match_reference(golden):
    arr = golden("gat3_train_grads.npz")
    m = _ref_model(GATRef, arr, "w.", dropout=0.0).train()
    x = torch.from_numpy(arr["x"]).requires_grad_(True)
    ei, y = torch.from_numpy(arr["edge_index"]), torch.from_numpy(arr["y"])
    logits = m(x, ei)
    mask = y != -1
    loss = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0]))(
        logits[mask].squeeze(1), y[mask].float())
    loss.backward()
    assert abs(loss.item() - float(arr["loss"])) < 1e-6 * max(1, abs(float(arr["loss"])))
    assert_close_scaled(x.grad, arr["grad_x"], rtol=1e-6, what="grad_x")
    for name, p in m.named_parameters():
        if not name.endswith("lin_dst.weight"):
            assert_close_scaled(p.grad, arr["grad." + name], rtol=1e-6, atol=1e-6, what=name)


def test_oracle_tgn_train_grads_match_reference(golden):
    """The TemporalGNN training step (tgn.py forward with h0 = 0, BCE(pos_weight
    = 50) on y != -1, backward) of the oracle wiring against the reference's own
    tgn.py run (tgn3_train_grads.npz)."""
    arr = golden("tgn3_train_grads.npz")
    m = _ref_model(TemporalGNNRef, arr, "w.", dropout=0.0).train()
    x = torch.from_numpy(arr["x"]).requires_grad_(True)
    ei, y = torch.from_numpy(arr["edge_index"]), torch.from_numpy(arr["y"])
    out, hid = m(x, ei)
    mask = y != -1
    loss = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0]))(
        out[mask].squeeze(1), y[mask].float())
    loss.backward()
    assert abs(loss.item() - float(arr["loss"])) < 1e-6 * max(1, abs(float(arr["loss"])))
    assert_close(hid, arr["hidden"], atol=1e-6, rtol=1e-6, what="hidden")
    assert_close_scaled(x.grad, arr["grad_x"], rtol=1e-6, what="grad_x")
    for name, p in m.named_parameters():
        if not name.endswith("lin_dst.weight"):
            assert_close_scaled(p.grad, arr["grad." + name], rtol=1e-6, atol=1e-6, what=name)


@pytest.mark.parametrize("fixture,case", [("gatconv_edgecases.npz", "base"),
                                          ("gatconv_edgecases.npz", "scale100"),
                                          ("gatconv_f166.npz", "pl")])
def test_oracle_single_layer_vectors(golden, fixture, case):
    arr = golden(fixture)
    t = lambda k: torch.from_numpy(arr[f"{case}.{k}"])  # noqa: E731
    out = gatconv_forward(t("x"), t("edge_index"), t("weight"), t("att_src"), t("att_dst"),
                          t("bias"))
    # these fixtures are the oracle's own outputs (make_golden.py): a regression
    # check of the restatement.  Not bit-exact across hosts: the CPU GEMM's
    # reduction order depends on the ISA / thread count (1 ulp observed between
    # an AVX-512 container and the one that wrote the fixtures).
    assert_close(out, arr[f"{case}.out"], atol=1e-6, rtol=1e-6, what=f"{fixture}/{case}")


def test_edgecase_fixture_covers_what_it_claims(golden):
    arr = golden("gatconv_edgecases.npz")
    ei = arr["base.edge_index"]
    N = arr["base.x"].shape[0]
    assert not (ei[1] == 0).any()                          # zero in-degree node
    assert (ei[0] == ei[1]).sum() >= 3                      # pre-existing self loops
    assert np.bincount(ei[1], minlength=N).max() >= 5000    # hub
    pairs = ei[0].astype(np.int64) * N + ei[1]
    assert len(np.unique(pairs)) < len(pairs)               # duplicates
    full = remove_then_add_self_loops(torch.from_numpy(ei), N)
    assert full.shape[1] == ei.shape[1] - (ei[0] == ei[1]).sum() + N


@pytest.mark.parametrize("fixture,case", [("gatconv_edgecases.npz", "base"),
                                          ("gatconv_f166.npz", "pl")])
def test_chunked_backward_oracle_matches_golden_grads(golden, fixture, case):
    """oracle.gatconv_grads_chunked (the large-graph backward checker: h once,
    destination chunks under autograd, dh summed) against the fixture grads of
    the plain PyG-dataflow autograd, with chunks small enough to split hubs'
    neighbourhoods across many chunk boundaries."""
    from oracle import gatconv_grads_chunked
    from _util import csr_cpu
    arr = golden(fixture)
    t = lambda k: torch.from_numpy(arr[f"{case}.{k}"])  # noqa: E731
    x = t("x")
    rp, col = csr_cpu(t("edge_index"), x.shape[0])
    r = gatconv_grads_chunked(x, rp, col, t("weight"), t("att_src"), t("att_dst"), t("bias"),
                              t("grad_out"), chunk_edges=997)
    for k in ("x", "weight", "att_src", "att_dst", "bias"):
        assert_close_scaled(r[k].reshape(arr[f"{case}.grad_{k}"].shape), arr[f"{case}.grad_{k}"],
                            rtol=2e-6, what=f"{fixture}/{case} grad_{k}")
