"""GPU parity of the reference model families on gfd's GATConv, against golden
vectors produced by the REFERENCE's own gat.py/tgn.py + shipped checkpoints
(tests/golden/make_golden.py)."""
import numpy as np
import pytest
import torch

from _util import assert_close, assert_close_scaled, state_dict_from

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(kind, arrays, prefix, in_ch=165, dropout=0.2):
    from gfd.models import GAT, TemporalGNN
    cls = GAT if kind == "gat" else TemporalGNN
    m = cls(in_channels=in_ch, hidden_channels=64, out_channels=1, num_layers=3, dropout=dropout)
    m.load_state_dict(state_dict_from(arrays, prefix), strict=True)
    return m.to(DEV)


def test_gat_checkpoint_eval_matches_reference(golden):
    arr = golden("elliptic_small.npz")
    m = _model("gat", arr, "gat.").eval()
    x = torch.from_numpy(arr["x"]).to(DEV)
    ei = torch.from_numpy(arr["edge_index"]).to(DEV)
    outs = []
    hooks = [c.register_forward_hook(lambda mod, i, o: outs.append(o)) for c in m.gat_layers]
    with torch.no_grad():
        logits = m(x, ei)
    for h in hooks:
        h.remove()
    for i, o in enumerate(outs):
        assert_close(o, arr[f"gat_layer{i}"], what=f"GATConv layer {i}")
    assert_close(logits, arr["gat_logits"], what="GAT logits")


def test_tgn_checkpoint_eval_matches_reference(golden):
    arr = golden("elliptic_small.npz")
    m = _model("tgn", arr, "tgn.").eval()
    x = torch.from_numpy(arr["x"]).to(DEV)
    ei = torch.from_numpy(arr["edge_index"]).to(DEV)
    with torch.no_grad():
        out, hid = m(x, ei)
        snap, _ = m.forward_snapshots(x, ei, torch.from_numpy(arr["time_step"]).to(DEV))
    assert_close(out, arr["tgn_out"], what="TGN out")
    assert_close(hid, arr["tgn_hidden"], what="TGN hidden")
    assert_close(snap, arr["tgn_out_snapshots"], what="TGN 49-step snapshots")


def test_gat_train_step_grads_match_reference(golden):
    """Config C2: fwd + BCE(pos_weight=50) + backward, dropout 0, train-mode BN."""
    arr = golden("gat3_train_grads.npz")
    m = _model("gat", arr, "w.", dropout=0.0).train()
    x = torch.from_numpy(arr["x"]).to(DEV).requires_grad_(True)
    ei = torch.from_numpy(arr["edge_index"]).to(DEV)
    y = torch.from_numpy(arr["y"]).to(DEV)
    logits = m(x, ei)
    mask = y != -1
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], device=DEV))
    loss = crit(logits[mask].squeeze(1), y[mask].float())
    loss.backward()
    assert_close(logits, arr["logits"], what="train logits")
    assert abs(loss.item() - float(arr["loss"])) <= 1e-4 * max(1.0, abs(float(arr["loss"])))
    assert_close_scaled(x.grad, arr["grad_x"], rtol=2e-4, what="grad_x")
    for name, p in m.named_parameters():
        if name.endswith("lin_dst.weight"):
            continue
        assert_close_scaled(p.grad, arr["grad." + name], rtol=2e-4, atol=1e-5, what=f"grad {name}")


def test_state_dict_roundtrip_keeps_lin_alias(golden):
    arr = golden("elliptic_small.npz")
    m = _model("gat", arr, "gat.")
    sd = m.state_dict()
    for i in range(3):
        assert sd[f"gat_layers.{i}.lin_src.weight"].data_ptr() == \
            sd[f"gat_layers.{i}.lin_dst.weight"].data_ptr()
    assert m.gat_layers[0].lin_dst is m.gat_layers[0].lin_src
