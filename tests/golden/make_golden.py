"""Generate the golden fixtures under tests/golden/ FROM THE REFERENCE ITSELF.

Runs only in the build container, where /root/reference exists (never on the
GPU box, never at test time).  Recipe:

1. inject the oracle ``GATConvRef`` (PyG-algorithm restatement) as
   ``torch_geometric.nn.GATConv`` -- PyG is not installed and cannot be;
2. import the reference's own ``src/models/gat.py`` and ``src/models/tgn.py``
   (no bytecode written: ``sys.dont_write_bytecode``);
3. load the shipped checkpoints ``results/{gat,tgn}_model.pt`` with
   ``torch.load(weights_only=True)`` and ``load_state_dict(strict=True)``;
4. run seeded synthetic graphs and write inputs, weights, per-layer outputs,
   logits and gradients as ``.npz`` data.

Only the data files are committed; no reference source or bytecode is.

    python tests/golden/make_golden.py
"""
from __future__ import annotations

import os
import sys
import types

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "gnn-fraud-detection_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from oracle.gatconv_ref import GATConvRef, gatconv_forward  # noqa: E402
from gfd import synth  # noqa: E402

# --- 1. shim PyG so the reference model code imports -------------------------
_tg = types.ModuleType("torch_geometric")
_tgnn = types.ModuleType("torch_geometric.nn")
_tgnn.GATConv = GATConvRef
_tg.nn = _tgnn
sys.modules["torch_geometric"] = _tg
sys.modules["torch_geometric.nn"] = _tgnn
sys.path.insert(0, REF)
from src.models.gat import GAT  # noqa: E402  (reference code, gat.py)
from src.models.tgn import TemporalGNN  # noqa: E402  (reference code, tgn.py)

torch.set_num_threads(8)


def load_ckpt(name):
    return torch.load(os.path.join(REF, "results", name), weights_only=True, map_location="cpu")


def sd_arrays(sd, prefix):
    out = {}
    for k, v in sd.items():
        if k.endswith("lin_dst.weight"):
            continue  # alias of lin_src.weight (same storage in the checkpoint)
        out[prefix + k] = v.detach().cpu().numpy()
    return out


def build_model(kind, sd, in_ch, dropout=0.2):
    cls = GAT if kind == "gat" else TemporalGNN
    m = cls(in_channels=in_ch, hidden_channels=64, out_channels=1, num_layers=3, dropout=dropout)
    m.load_state_dict(sd, strict=True)
    return m


def capture_layers(model):
    outs = []
    hooks = [g.register_forward_hook(lambda mod, inp, out: outs.append(out.detach().clone()))
             for g in model.gat_layers]
    return outs, hooks


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {name}: {os.path.getsize(path) / 1e6:.2f} MB, keys={sorted(arrays)[:6]}...")


def elliptic_small():
    g = synth.elliptic_like(num_nodes=1500, num_edges=1725, num_steps=49, num_features=165, seed=0)
    x = torch.from_numpy(g["x"])
    ei = torch.from_numpy(g["edge_index"])
    arrays = {"x": g["x"], "edge_index": g["edge_index"], "time_step": g["time_step"], "y": g["y"]}
    sd_gat, sd_tgn = load_ckpt("gat_model.pt"), load_ckpt("tgn_model.pt")
    arrays.update(sd_arrays(sd_gat, "gat."))
    arrays.update(sd_arrays(sd_tgn, "tgn."))
    gat = build_model("gat", sd_gat, 165).eval()
    outs, hooks = capture_layers(gat)
    with torch.no_grad():
        logits = gat(x, ei)
    for h in hooks:
        h.remove()
    for i, o in enumerate(outs):
        arrays[f"gat_layer{i}"] = o.numpy()
    arrays["gat_logits"] = logits.numpy()
    tgn = build_model("tgn", sd_tgn, 165).eval()
    outs, hooks = capture_layers(tgn)
    with torch.no_grad():
        out, hid = tgn(x, ei)
    for h in hooks:
        h.remove()
    arrays["tgn_out"] = out.numpy()
    arrays["tgn_hidden"] = hid.numpy()
    # per-time-step snapshots (config C3): step forward on each induced subgraph, h0 = 0
    ts = g["time_step"]
    snap = np.zeros_like(arrays["tgn_out"])
    with torch.no_grad():
        for s in range(1, 50):
            idx = np.nonzero(ts == s)[0]
            lo = idx[0]
            m = (ts[g["edge_index"][1]] == s)
            sub_ei = torch.from_numpy(g["edge_index"][:, m] - lo)
            o, _ = tgn(x[idx[0]:idx[-1] + 1], sub_ei)
            snap[idx] = o.numpy()
    arrays["tgn_out_snapshots"] = snap
    save("elliptic_small.npz", **arrays)


def train_grads():
    g = synth.elliptic_like(num_nodes=1000, num_edges=1150, num_steps=49, num_features=165, seed=3)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    ei = torch.from_numpy(g["edge_index"])
    y = torch.from_numpy(g["y"])
    sd = load_ckpt("gat_model.pt")
    gat = build_model("gat", sd, 165, dropout=0.0).train()
    logits = gat(x, ei)                                           # train.py:124
    mask = y != -1                                                # train.py:108
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0]))  # train.py:360-361
    loss = crit(logits[mask].squeeze(1), y[mask].float())        # train.py:139
    loss.backward()                                               # train.py:142
    arrays = {"x": g["x"], "edge_index": g["edge_index"], "y": g["y"],
              "logits": logits.detach().numpy(), "loss": np.array(loss.item(), dtype=np.float64),
              "grad_x": x.grad.numpy()}
    arrays.update(sd_arrays(sd, "w."))
    for name, p in gat.named_parameters():
        if name.endswith("lin_dst.weight"):
            continue
        arrays["grad." + name] = p.grad.numpy()
    save("gat3_train_grads.npz", **arrays)


def tgn_train_grads():
    """One training step of the reference's TemporalGNN (train.py:115-121 runs
    the same loop for --model_type tgn): tgn.py forward with h0 = 0 (the
    GRUCell(h, 0) + Linear head, tgn.py:88-89, 108-111), BCE(pos_weight=50)
    on the labelled nodes, backward.  Dropout 0 so the step is deterministic."""
    g = synth.elliptic_like(num_nodes=1000, num_edges=1150, num_steps=49, num_features=165, seed=4)
    x = torch.from_numpy(g["x"]).requires_grad_(True)
    ei = torch.from_numpy(g["edge_index"])
    y = torch.from_numpy(g["y"])
    sd = load_ckpt("tgn_model.pt")
    tgn = build_model("tgn", sd, 165, dropout=0.0).train()
    out, hidden = tgn(x, ei)                                      # train.py:117 (tgn branch)
    mask = y != -1
    crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0]))
    loss = crit(out[mask].squeeze(1), y[mask].float())
    loss.backward()
    arrays = {"x": g["x"], "edge_index": g["edge_index"], "y": g["y"],
              "logits": out.detach().numpy(), "hidden": hidden.detach().numpy(),
              "loss": np.array(loss.item(), dtype=np.float64), "grad_x": x.grad.numpy()}
    arrays.update(sd_arrays(sd, "w."))
    for name, p in tgn.named_parameters():
        if name.endswith("lin_dst.weight"):
            continue
        arrays["grad." + name] = p.grad.numpy()
    save("tgn3_train_grads.npz", **arrays)


def single_layer_case(name, x, ei, seed, att_scale=1.0):
    gen = torch.Generator().manual_seed(seed)
    conv = GATConvRef(x.shape[1], 64, heads=8, concat=False, dropout=0.0)
    conv.reset_parameters(gen)
    with torch.no_grad():
        conv.att_src.mul_(att_scale)
        conv.att_dst.mul_(att_scale)
        conv.bias.copy_(torch.randn(64, generator=gen) * 0.1)
    xt = torch.from_numpy(x).requires_grad_(True)
    out, st = gatconv_forward(xt, torch.from_numpy(ei), conv.lin_src.weight, conv.att_src,
                              conv.att_dst, conv.bias, heads=8, return_stats=True)
    gout = torch.randn(out.shape, generator=gen)
    (out * gout).sum().backward()
    return {f"{name}.x": x, f"{name}.edge_index": ei,
            f"{name}.weight": conv.lin_src.weight.detach().numpy(),
            f"{name}.att_src": conv.att_src.detach().numpy(),
            f"{name}.att_dst": conv.att_dst.detach().numpy(),
            f"{name}.bias": conv.bias.detach().numpy(),
            f"{name}.out": out.detach().numpy(), f"{name}.grad_out": gout.numpy(),
            f"{name}.max": st["max"].numpy(), f"{name}.sum": st["sum"].numpy(),
            f"{name}.grad_x": xt.grad.numpy(),
            f"{name}.grad_weight": conv.lin_src.weight.grad.numpy(),
            f"{name}.grad_att_src": conv.att_src.grad.numpy(),
            f"{name}.grad_att_dst": conv.att_dst.grad.numpy(),
            f"{name}.grad_bias": conv.bias.grad.numpy()}


def edge_cases():
    rng = np.random.Generator(np.random.PCG64(7))
    N, F = 300, 166
    x = rng.standard_normal((N, F), dtype=np.float32)
    src = rng.integers(0, N, 900)
    dst = rng.integers(0, N, 900)
    dst[dst == 0] = 1                       # node 0: zero in-degree (self loop only)
    loops = np.array([[3, 7, 11], [3, 7, 11]])          # pre-existing self loops (dropped, re-added)
    dup = np.array([[20, 20, 20, 21], [22, 22, 22, 22]])  # duplicate edges (kept)
    hub_src = rng.integers(0, N, 5000)
    hub = np.stack([hub_src, np.full(5000, 5)])         # hub: in-degree 5000
    ei = np.concatenate([np.stack([src, dst]), loops, dup, hub], axis=1).astype(np.int64)
    ei = ei[:, rng.permutation(ei.shape[1])]
    arrays = {}
    arrays.update(single_layer_case("base", x, ei, seed=11))
    arrays.update(single_layer_case("scale100", x, ei, seed=12, att_scale=100.0))
    save("gatconv_edgecases.npz", **arrays)


def f166_powerlaw():
    ei = synth.power_law(2048, 10000, seed=5)
    x = np.random.Generator(np.random.PCG64(5)).standard_normal((2048, 166), dtype=np.float32)
    save("gatconv_f166.npz", **single_layer_case("pl", x, ei, seed=13))


if __name__ == "__main__":
    which = sys.argv[1:] or ["elliptic_small", "train_grads", "tgn_train_grads", "edge_cases",
                             "f166_powerlaw"]
    for fn in which:
        globals()[fn]()
