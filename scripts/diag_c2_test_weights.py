"""Where does grad_x of the Adam-weights C2 test (tests/test_fullsize_models_gpu.py::
test_c2_full_size_train_step_at_adam_updated_weights) differ from fp64?  Reproduces
the test's weights, then reports the largest |device - fp64| grad_x rows and, for those
nodes, the smallest |pre-ReLU value| of each layer in the fp64 forward (a ReLU flip
shows as a near-zero pre-activation).

usage: python scripts/diag_c2_test_weights.py
"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import torch  # noqa: E402

from gfd import synth  # noqa: E402
from gfd.models import GAT  # noqa: E402
from oracle import GATRef  # noqa: E402

DEV = "cuda"
d = synth.elliptic_like(num_features=165, seed=0)
torch.manual_seed(0)
m = GAT(165, 64, 1, num_layers=3, dropout=0.2).to(DEV).train()
y = torch.from_numpy(d["y"])
mask = y != -1
yl = y[mask].float()
xd = torch.from_numpy(d["x"]).to(DEV)
eid = torch.from_numpy(d["edge_index"]).to(DEV)
md, yld = mask.to(DEV), yl.to(DEV)
opt = torch.optim.Adam(m.parameters(), lr=1e-3, weight_decay=5e-4)
crit = torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], device=DEV))
for _ in range(12):
    opt.zero_grad()
    crit(m(xd, eid)[md].squeeze(1), yld).backward()
    opt.step()
sd = {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}
g = GAT(165, 64, 1, num_layers=3, dropout=0.0)
g.load_state_dict(sd, strict=True)
g = g.to(DEV).train()
x = xd.clone().requires_grad_(True)
crit(g(x, eid)[md].squeeze(1), yld).backward()
gx = x.grad.detach().cpu().double()

ref = GATRef(165, 64, 1, num_layers=3, dropout=0.0).train()
ref.load_state_dict(sd, strict=True)
ref = ref.double()
pre = {}
for i, bn in enumerate(ref.batch_norms):
    bn.register_forward_hook(lambda mod, inp, out, i=i: pre.__setitem__(i, out.detach()))
xr = torch.from_numpy(d["x"]).double().requires_grad_(True)
rl = ref(xr, torch.from_numpy(d["edge_index"]))
torch.nn.BCEWithLogitsLoss(pos_weight=torch.tensor([50.0], dtype=torch.float64))(
    rl[mask].squeeze(1), yl.double()).backward()
err = (gx - xr.grad).abs().max(1).values
top = torch.topk(err, 8)
print("max|grad_x| fp64", xr.grad.abs().max().item(), "max err", err.max().item())
ei = torch.from_numpy(d["edge_index"])
for e, n in zip(top.values.tolist(), top.indices.tolist()):
    nb = torch.cat([torch.tensor([n]), ei[1][ei[0] == n], ei[0][ei[1] == n]]).unique()
    mins = [round(pre[i][nb].abs().min().item(), 9) for i in sorted(pre)]
    print(f"node {n}: err {e:.3e}; min |pre-ReLU| over it and its neighbours per layer {mins}")
