"""Dump GPU gradients of the C2 train-step fixture (for fp64 comparison on the host)."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "tests"), os.path.join(REPO, "gnn-fraud-detection_amd")]
import numpy as np, torch
from conftest import load_golden
from _util import state_dict_from
from gfd.models import GAT
arr = load_golden("gat3_train_grads.npz")
m = GAT(165, 64, 1, num_layers=3, dropout=0.0)
m.load_state_dict(state_dict_from(arr, "w."), strict=True)
m = m.cuda().train()
x = torch.from_numpy(arr["x"]).cuda().requires_grad_(True)
ei = torch.from_numpy(arr["edge_index"]).cuda(); y = torch.from_numpy(arr["y"]).cuda()
acts = {}
for i, c in enumerate(m.gat_layers):
    def fh(mod, inp, out, i=i):
        acts[f"in{i}"] = inp[0].detach().cpu().numpy()
        acts[f"out{i}"] = out.detach().cpu().numpy()
    def bh(mod, gi, go, i=i):
        acts[f"gout{i}"] = go[0].detach().cpu().numpy()
    c.register_forward_hook(fh)
    c.register_full_backward_hook(bh)
lg = m(x, ei); mask = y != -1
loss = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], device="cuda"))(lg[mask].squeeze(1), y[mask].float())
loss.backward()
out = {"grad_x": x.grad.cpu().numpy()}
for n, p in m.named_parameters():
    out["grad." + n] = p.grad.cpu().numpy()
out.update(acts)
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "diag_grads.npz"), **out)
print("saved", len(out))
