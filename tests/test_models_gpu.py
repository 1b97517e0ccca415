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
    hooks = [c.register_forward_hook(lambda mod, i, o: outs.append(o.detach())) for c in m.gat_layers]
    logits_unfused = m(x, ei).detach()     # grad enabled: GATConv -> ATen BN/ReLU/residual
    for h in hooks:
        h.remove()
    assert len(outs) == 3
    for i, o in enumerate(outs):
        assert_close(o, arr[f"gat_layer{i}"], what=f"GATConv layer {i}")
    assert_close(logits_unfused, arr["gat_logits"], what="GAT logits (unfused)")
    with torch.no_grad():                  # inference: fused layer epilogues
        logits = m(x, ei)
    assert_close(logits, arr["gat_logits"], what="GAT logits (fused epilogues)")


def test_tgn_checkpoint_eval_matches_reference(golden):
    arr = golden("elliptic_small.npz")
    m = _model("tgn", arr, "tgn.").eval()
    x = torch.from_numpy(arr["x"]).to(DEV)
    ei = torch.from_numpy(arr["edge_index"]).to(DEV)
    with torch.no_grad():                  # fused layer epilogues + fused GRU/Linear head
        out, hid = m(x, ei)
        snap, _ = m.forward_snapshots(x, ei, torch.from_numpy(arr["time_step"]).to(DEV))
    assert_close(out, arr["tgn_out"], what="TGN out")
    assert_close(hid, arr["tgn_hidden"], what="TGN hidden")
    assert_close(snap, arr["tgn_out_snapshots"], what="TGN 49-step snapshots")
    out_u, hid_u = m(x, ei)                # grad enabled: unfused path
    assert_close(out_u.detach(), arr["tgn_out"], what="TGN out (unfused)")
    assert_close(hid_u.detach(), arr["tgn_hidden"], what="TGN hidden (unfused)")


@pytest.mark.parametrize("residual,relu,dtype", [(True, True, torch.float32),
                                                 (False, True, torch.float32),
                                                 (True, False, torch.bfloat16)])
def test_fused_layer_epilogue_matches_unfused(residual, relu, dtype):
    """gfd.fused.gat_layer (BN / ReLU / residual applied in the GATConv store
    epilogue) against the same GATConv followed by ATen ops, with non-trivial
    BatchNorm running statistics, on a graph with hubs, light and lone rows."""
    from gfd import fused, synth
    from gfd.nn import GATConv
    torch.manual_seed(5)
    N = 20000
    ei = torch.from_numpy(synth.power_law(N, 160000, seed=5)).to(DEV)
    x = torch.randn(N, 64, device=DEV).to(dtype)
    conv = GATConv(64, 64, heads=8, concat=False).to(DEV)
    with torch.no_grad():
        conv.bias.normal_()
    bn = torch.nn.BatchNorm1d(64).to(DEV).eval()
    with torch.no_grad():
        bn.running_mean.normal_()
        bn.running_var.uniform_(0.5, 2.0)
        bn.weight.normal_()
        bn.bias.normal_()
        ref = bn(conv(x, ei))
        if relu:
            ref = torch.relu(ref)
        if residual:
            ref = ref + x.float()
        got = fused.gat_layer(conv, bn, x, ei, relu=relu, residual=residual)
    assert_close(got, ref, what=f"fused layer residual={residual} relu={relu} {dtype}")


@pytest.mark.parametrize("with_h0", [False, True])
def test_fused_gru_head_matches_torch(with_h0):
    from gfd import fused
    torch.manual_seed(6)
    gru = torch.nn.GRUCell(64, 64).to(DEV)
    lin = torch.nn.Linear(64, 3).to(DEV)
    h = torch.randn(5003, 64, device=DEV)
    h0 = torch.randn(5003, 64, device=DEV) if with_h0 else None
    with torch.no_grad():
        hr = gru(h, h0 if h0 is not None else torch.zeros_like(h))
        outr = lin(hr)
        out, hn = fused.gru_head(gru, lin, h, h0)
    assert_close(hn, hr, what="GRUCell h'")
    assert_close(out, outr, what="Linear head")


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
