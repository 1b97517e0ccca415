"""Diagnose the 2M-node backward parity: GPU grads vs fp32 and fp64 chunked
oracles, error by grad_W row group (head channels / ds / dt)."""
import os, sys, time
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import torch
import bench
from gfd.nn import gat_conv
from oracle import gatconv_grads_chunked

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
E = 5 * N
DEV = torch.device("cuda", 0)
s = bench.setup(DEV, N, E, 166)
g = s["graph"]
g.csc()
gen = torch.Generator().manual_seed(6)
bias = (torch.randn(64, generator=gen) * 0.1).to(DEV)
x = s["x"].detach().requires_grad_(True)
W = s["W"].clone().requires_grad_(True)
a_s = s["a_s"].clone().requires_grad_(True)
a_d = s["a_d"].clone().requires_grad_(True)
b = bias.clone().requires_grad_(True)
gout = torch.randn((g.num_nodes, 64), generator=gen)
out = gat_conv(x, g, W, a_s, a_d, b, training=True)
out.backward(gout.to(DEV))
torch.cuda.synchronize()
got = {"x": x.grad.cpu().double(), "weight": W.grad.cpu().double(), "att_src": a_s.grad.cpu().double().reshape(1, 8, 64),
       "att_dst": a_d.grad.cpu().double().reshape(1, 8, 64), "bias": b.grad.cpu().double()}
t0 = time.time()
r64 = gatconv_grads_chunked(s["x"].detach().cpu(), g.rowptr.cpu(), g.col.cpu(), s["W"].cpu(), s["a_s"].cpu(),
                            s["a_d"].cpu(), bias.cpu(), gout, dtype=torch.float64)
print("oracle64", time.time() - t0, flush=True)
r32 = gatconv_grads_chunked(s["x"].detach().cpu(), g.rowptr.cpu(), g.col.cpu(), s["W"].cpu(), s["a_s"].cpu(),
                            s["a_d"].cpu(), bias.cpu(), gout)
for k in ("weight", "att_src", "att_dst", "bias", "x"):
    ref = r64[k].reshape(got[k].shape)
    e_gpu = (got[k] - ref).abs()
    e_32 = (r32[k].double().reshape(ref.shape) - ref).abs()
    print(k, "scale", ref.abs().max().item(), "gpu err", e_gpu.max().item(), "fp32-oracle err", e_32.max().item(), flush=True)
ref = r64["weight"]
e = (got["weight"] - ref).abs()
print("grad_W err per head (rows h*64..):", [round(e[h * 64:(h + 1) * 64].max().item(), 5) for h in range(8)])
print("grad_W err per feature (top 10):", torch.topk(e.max(0).values, 10))
print("grad_W ref col scale (top 5):", torch.topk(ref.abs().max(0).values, 5))
rel = (e.max(0).values / ref.abs().max(0).values)
print("per-column relative err max", rel.max().item(), "median", rel.median().item())
# dh' dynamic range proxy: out-degree
cp = g.csc().colptr.long()
od = cp[1:] - cp[:-1]
print("max out-degree", od.max().item(), "max in-degree", (g.rowptr[1:] - g.rowptr[:-1]).max().item())
