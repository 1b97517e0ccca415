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


@pytest.mark.parametrize("residual,relu", [(True, True), (False, True), (True, False)])
def test_train_body_matches_torch(residual, relu):
    """gfd.fused.train_body (batch-statistics BN -> ReLU -> residual, dropout 0)
    against torch.nn.BatchNorm1d(train) + ATen: output, running statistics,
    and the gradients of y, the residual input, gamma and beta."""
    from gfd import fused
    torch.manual_seed(8)
    N = 30011
    y0 = (torch.randn(N, 64, device=DEV) * 3 + 1).requires_grad_(True)
    h0 = torch.randn(N, 64, device=DEV).requires_grad_(True)
    bn_r = torch.nn.BatchNorm1d(64).to(DEV).train()
    with torch.no_grad():
        bn_r.weight.normal_()
        bn_r.bias.normal_()
    bn_g = torch.nn.BatchNorm1d(64).to(DEV).train()
    bn_g.load_state_dict(bn_r.state_dict())
    ref = bn_r(y0)
    ref = torch.relu(ref) if relu else ref
    ref = ref + h0 if residual else ref
    g = torch.randn_like(ref)
    gr = torch.autograd.grad(ref, [y0, h0, bn_r.weight, bn_r.bias], g, allow_unused=True)
    y1 = y0.detach().clone().requires_grad_(True)
    h1 = h0.detach().clone().requires_grad_(True)
    got = fused.train_body(y1, bn_g, h1 if residual else None, relu=relu, p=0.0)
    gg = torch.autograd.grad(got, [y1, h1, bn_g.weight, bn_g.bias], g, allow_unused=True)
    assert_close(got, ref, what="train body out")
    assert_close(bn_g.running_mean, bn_r.running_mean, what="running_mean")
    assert_close(bn_g.running_var, bn_r.running_var, what="running_var")
    assert int(bn_g.num_batches_tracked) == int(bn_r.num_batches_tracked) == 1
    names = ["grad y", "grad residual", "grad gamma", "grad beta"]
    for a, b, nm in zip(gg, gr, names):
        if b is None:
            assert a is None, nm
        else:
            assert_close_scaled(a, b, rtol=1e-4, what=nm)


def test_train_body_dropout_mask():
    """p > 0: the kept fraction is 1 - p, kept entries are scaled by 1/(1-p),
    the same seed gives the same mask, and the backward uses that mask."""
    from gfd import fused
    torch.manual_seed(9)
    N, p = 40000, 0.2
    y = torch.randn(N, 64, device=DEV).requires_grad_(True)
    bn = torch.nn.BatchNorm1d(64).to(DEV).train()
    torch.manual_seed(10)
    out = fused.train_body(y, bn, None, relu=False, p=p)
    torch.manual_seed(10)
    out2 = fused.train_body(y, torch.nn.BatchNorm1d(64).to(DEV).train(), None, relu=False, p=p)
    assert torch.equal(out, out2)
    with torch.no_grad():
        z = torch.nn.functional.batch_norm(y, None, None, bn.weight, bn.bias, True, 0.0, bn.eps)
    keep = out != 0
    frac = keep.float().mean().item()
    assert abs(frac - (1 - p)) < 0.005, frac
    assert_close(out[keep], (z / (1 - p))[keep], what="kept entries")
    g = torch.randn_like(out)
    (gy,) = torch.autograd.grad(out, [y], g)
    yr = y.detach().clone().requires_grad_(True)
    zr = torch.nn.functional.batch_norm(yr, None, None, bn.weight.detach(), bn.bias.detach(),
                                        True, 0.0, bn.eps)
    (gr,) = torch.autograd.grad(zr * keep.float() / (1 - p), [yr], g)
    assert_close_scaled(gy, gr, rtol=1e-4, what="dropout backward")


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


def test_tgn_train_step_grads_match_reference(golden):
    """The TemporalGNN training step (train.py:115-121, 139-142 for the tgn
    model): GAT stack + GRUCell(h, 0) + Linear in training mode on the device
    (gfd.fused.tgn_head_train: one kernel forward, one backward), BCE(pos_weight
    = 50), backward -- every gradient against the reference's own tgn.py run."""
    arr = golden("tgn3_train_grads.npz")
    m = _model("tgn", arr, "w.", dropout=0.0).train()
    x = torch.from_numpy(arr["x"]).to(DEV).requires_grad_(True)
    ei = torch.from_numpy(arr["edge_index"]).to(DEV)
    y = torch.from_numpy(arr["y"]).to(DEV)
    out, hid = m(x, ei)
    mask = y != -1
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], device=DEV))
    loss = crit(out[mask].squeeze(1), y[mask].float())
    loss.backward()
    assert_close(out, arr["logits"], what="tgn train logits")
    assert_close(hid, arr["hidden"], what="tgn train hidden")
    assert abs(loss.item() - float(arr["loss"])) <= 1e-4 * max(1.0, abs(float(arr["loss"])))
    assert_close_scaled(x.grad, arr["grad_x"], rtol=2e-4, what="grad_x")
    for name, p in m.named_parameters():
        if name.endswith("lin_dst.weight"):
            continue
        assert_close_scaled(p.grad, arr["grad." + name], rtol=2e-4, atol=1e-5, what=f"grad {name}")


def test_tgn_head_train_kernel_matches_autograd():
    """gfd.fused.tgn_head_train (GRUCell + Linear forward and backward kernels)
    against torch autograd of nn.GRUCell + nn.Linear in fp64, with and without
    h0, with a gradient on the hidden output too, rows not a multiple of 16."""
    from gfd.fused import tgn_head_train
    torch.manual_seed(0)
    gru = torch.nn.GRUCell(64, 64).to(DEV)
    lin = torch.nn.Linear(64, 1).to(DEV)
    for N, with_h0 in ((1000, False), (4099, True)):
        h = torch.randn(N, 64, device=DEV, requires_grad=True)
        h0 = torch.randn(N, 64, device=DEV, requires_grad=True) if with_h0 else None
        go = torch.randn(N, 1, device=DEV)
        gh = torch.randn(N, 64, device=DEV) * 0.1
        out, hn = tgn_head_train(gru, lin, h, h0)
        (out * go).sum().add_((hn * gh).sum()).backward()
        got = {"h": h.grad.clone(), "w_ih": gru.weight_ih.grad.clone(),
               "w_hh": gru.weight_hh.grad.clone(), "b_ih": gru.bias_ih.grad.clone(),
               "b_hh": gru.bias_hh.grad.clone(), "w_o": lin.weight.grad.clone(),
               "b_o": lin.bias.grad.clone()}
        if with_h0:
            got["h0"] = h0.grad.clone()
        for p in list(gru.parameters()) + list(lin.parameters()):
            p.grad = None
        g64 = torch.nn.GRUCell(64, 64).double().to(DEV)
        l64 = torch.nn.Linear(64, 1).double().to(DEV)
        g64.load_state_dict({k: v.double() for k, v in gru.state_dict().items()})
        l64.load_state_dict({k: v.double() for k, v in lin.state_dict().items()})
        hr = h.detach().double().requires_grad_(True)
        h0r = h0.detach().double().requires_grad_(True) if with_h0 else None
        hnr = g64(hr, h0r)
        outr = l64(hnr)
        (outr * go.double()).sum().add_((hnr * gh.double()).sum()).backward()
        assert_close(out, outr, what="tgn head out")
        assert_close(hn, hnr, what="tgn head hidden")
        want = {"h": hr.grad, "w_ih": g64.weight_ih.grad, "w_hh": g64.weight_hh.grad,
                "b_ih": g64.bias_ih.grad, "b_hh": g64.bias_hh.grad, "w_o": l64.weight.grad,
                "b_o": l64.bias.grad}
        if with_h0:
            want["h0"] = h0r.grad
        for k in want:
            assert_close_scaled(got[k], want[k], rtol=1e-5, what=f"N={N} h0={with_h0} grad {k}")
        h.grad = None


def test_state_dict_roundtrip_keeps_lin_alias(golden):
    arr = golden("elliptic_small.npz")
    m = _model("gat", arr, "gat.")
    sd = m.state_dict()
    for i in range(3):
        assert sd[f"gat_layers.{i}.lin_src.weight"].data_ptr() == \
            sd[f"gat_layers.{i}.lin_dst.weight"].data_ptr()
    assert m.gat_layers[0].lin_dst is m.gat_layers[0].lin_src


@pytest.mark.parametrize("layers,F", [(3, 165), (1, 166)])
def test_gat_head_folded_into_last_layer_store(layers, F):
    """Inference: the GAT head Linear(64, 1) (gat.py:94) folded into the last
    layer's store (gfd_epilogue.head_*: a row dot in the tile / lone / logits
    kernels instead of writing [N, 64] and re-reading it) against the body
    written out and the head applied by ATen, on a graph with hubs, general,
    light and self-loop-only rows."""
    from gfd import synth
    from gfd.models import GAT
    torch.manual_seed(11)
    N = 20000
    ei = torch.from_numpy(synth.power_law(N, 160000, seed=11)).to(DEV)
    x = torch.randn(N, F, device=DEV)
    m = GAT(F, 64, 1, num_layers=layers).to(DEV).eval()
    with torch.no_grad():
        for bn in m.batch_norms:
            bn.running_mean.normal_()
            bn.running_var.uniform_(0.5, 2.0)
        for conv in m.gat_layers:
            conv.bias.normal_()
        m.out.bias.normal_()
        folded = m(x, ei)
        body = m.encode(x, ei)
        want = body @ m.out.weight.t() + m.out.bias
    assert folded.shape == (N, 1)
    assert_close(folded, want, what=f"folded head, {layers} layers")


def test_gat_inference_with_slope_outside_unit_interval():
    """negative_slope outside [0, 1] takes the k_fused path, which cannot fold
    the head: GAT.forward must not try and still match the body
    written out plus the head applied by ATen, and the oracle."""
    from gfd import synth
    from gfd.models import GAT
    from oracle import GATRef
    torch.manual_seed(12)
    N, F = 3000, 165
    ei = torch.from_numpy(synth.power_law(N, 20000, seed=12))
    x = torch.randn(N, F)
    ref = GATRef(F, 64, 1, num_layers=2).eval()
    for conv in ref.gat_layers:
        conv.negative_slope = 1.5
    m = GAT(F, 64, 1, num_layers=2).to(DEV).eval()
    m.load_state_dict(ref.state_dict(), strict=True)
    for conv in m.gat_layers:
        conv.negative_slope = 1.5
    with torch.no_grad():
        got = m(x.to(DEV), ei.to(DEV))
        want = ref(x, ei)
        body = m.encode(x.to(DEV), ei.to(DEV))
    assert got.shape == (N, 1)
    assert_close(got, want, what="GAT, slope 1.5")
    assert_close(got, body @ m.out.weight.t() + m.out.bias, what="GAT, slope 1.5, unfolded head")
