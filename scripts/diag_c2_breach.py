"""Per-tensor C2 gradient parity at the bench leg's weights.

Reproduces bench_legs.c2_gat3_train_step's weights (seed-0 init, the leg's
warm-up + timed Adam steps at dropout 0.2), then one dropout-0 fwd + BCE + bwd
step on the device, in the fp32 oracle and in an fp64 oracle.  Prints, per
tensor, max |err| of the device and of the fp32 oracle against fp64, and saves
the state dict and every gradient to gpurun_out/diag_c2.npz.

usage: python scripts/diag_c2_breach.py [adam_steps]
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench_legs  # noqa: E402
from gfd.models import GAT  # noqa: E402
from oracle import GATRef  # noqa: E402

dev = "cuda"
steps = int(sys.argv[1]) if len(sys.argv) > 1 else 23
d = bench_legs._elliptic(dev)
m = bench_legs._model("gat", 165, 3, dev).train()
opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=5e-4)
crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], device=dev))
mask = d["y"] != -1
yl = d["y"][mask].float()
for _ in range(steps):
    opt.zero_grad()
    loss = crit(m(d["x"], d["edge_index"])[mask].squeeze(1), yl)
    loss.backward()
    opt.step()
torch.cuda.synchronize()
sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}

g = GAT(165, 64, 1, num_layers=3, dropout=0.0)
g.load_state_dict(sd, strict=True)
g = g.to(dev).train()
x = d["x"].clone().requires_grad_(True)
lg = g(x, d["edge_index"])
crit(lg[mask].squeeze(1), yl).backward()
torch.cuda.synchronize()
gpu = {"x": x.grad.cpu().double()}
gpu.update({n: p.grad.cpu().double() for n, p in g.named_parameters() if p.grad is not None})


def oracle(dtype):
    r = GATRef(165, 64, 1, num_layers=3, dropout=0.0).train()
    r.load_state_dict(sd, strict=True)
    r = r.to(dtype)
    xr = d["x"].cpu().to(dtype).requires_grad_(True)
    lr = r(xr, d["edge_index"].cpu())
    torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], dtype=dtype))(
        lr[mask.cpu()].squeeze(1), yl.cpu().to(dtype)).backward()
    out = {"x": xr.grad.double()}
    out.update({n: p.grad.double() for n, p in r.named_parameters() if p.grad is not None})
    return out, lr.detach().double()


r32, l32 = oracle(torch.float32)
r64, l64 = oracle(torch.float64)
print(f"adam steps {steps}; logits max|gpu-f64| {(lg.detach().cpu().double() - l64).abs().max():.3e} "
      f"max|f32-f64| {(l32 - l64).abs().max():.3e}")
print(f"{'tensor':34s} {'max|ref64|':>11s} {'gpu-f64':>10s} {'f32-f64':>10s} {'gpu-f32':>10s} "
      f"{'gpu/bound':>9s} {'f32/bound':>9s}")
save = {}
for n in gpu:
    if n.endswith("lin_dst.weight"):
        continue
    a, b, c = gpu[n], r32[n], r64[n]
    den = c.abs().max().item()
    bound = 2e-4 * den + 1e-5
    e_g, e_3, e_g3 = (a - c).abs().max().item(), (b - c).abs().max().item(), (a - b).abs().max().item()
    print(f"{n:34s} {den:11.3e} {e_g:10.3e} {e_3:10.3e} {e_g3:10.3e} {e_g / bound:9.3f} {e_3 / bound:9.3f}")
    save["gpu." + n], save["f32." + n], save["f64." + n] = a.numpy(), b.numpy(), c.numpy()
for k, v in sd.items():
    save["w." + k] = v.numpy()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "diag_c2.npz"), **save)
print("saved gpurun_out/diag_c2.npz")
