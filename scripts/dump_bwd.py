"""Dump one GATConv forward + backward (grad_x, grad_W, grad_att, grad_bias) on
a seeded power-law graph for the library named by GFD_LIB_PATH, into
gpurun_out/<tag>.npz (A/B of backward kernel variants: compare two dumps with
scripts/cmp_dumps.py; the deterministic backward makes them bit-identical when
the arithmetic is)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402
from gfd import synth  # noqa: E402
from gfd.nn import gat_conv  # noqa: E402

tag = sys.argv[1]
N, E, F, H, C = 400_000, 3_000_000, 166, 8, 64
dev = "cuda"
gen = torch.Generator().manual_seed(5)
ei = torch.from_numpy(synth.power_law(N, E, seed=5)).to(dev)
x = torch.randn(N, F, generator=gen).to(dev).requires_grad_(True)
W = (torch.randn(H * C, F, generator=gen) * 0.08).to(dev).requires_grad_(True)
a_s = (torch.randn(1, H, C, generator=gen) * 0.1).to(dev).requires_grad_(True)
a_d = (torch.randn(1, H, C, generator=gen) * 0.1).to(dev).requires_grad_(True)
b = (torch.randn(C, generator=gen) * 0.1).to(dev).requires_grad_(True)
g = torch.randn(N, C, generator=gen).to(dev)
out = gat_conv(x, ei, W, a_s, a_d, b)
(out * g).sum().backward()
torch.cuda.synchronize()
res = {"out": out.detach().cpu().numpy()}
for k, t in (("x", x), ("W", W), ("att_src", a_s), ("att_dst", a_d), ("bias", b)):
    res["grad_" + k] = t.grad.cpu().numpy()
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", f"{tag}.npz"), **res)
print("saved", tag, {k: v.shape for k, v in res.items()})
