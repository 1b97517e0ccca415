"""Trace one node's backward inputs: for node j, every destination i of its
out-messages -- forward stats (max, sum per head), alpha~ / dpre per message
and dt_i from the GPU workspace -- against fp64 recomputation."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import torch
import torch.nn.functional as Fn
import bench
from gfd import _lib

N = int(sys.argv[1]); nodes = [int(v) for v in sys.argv[2].split(",")]
DEV = torch.device("cuda", 0)
s = bench.setup(DEV, N, 5 * N, 166)
g = s["graph"]; csc = g.csc(); plan, splan = g.plan(), csc.plan
F, H, C = 166, 8, 64
gen = torch.Generator().manual_seed(6)
bias = (torch.randn(64, generator=gen) * 0.1).to(DEV)
gout = torch.randn((N, 64), generator=gen)
x = s["x"]
out = torch.empty((N, C), device=DEV); st = torch.empty((N, 16), device=DEV); stats = torch.empty((N, 16), device=DEV)
lib = _lib.load()
ws = torch.empty(lib.gfd_gat_fwd_workspace_size(N, N, F, H, C, plan.num_hubs, plan.num_chunks), dtype=torch.uint8, device=DEV)
_lib.call("gfd_gat_fwd", x.data_ptr(), 0, N, F, x.stride(0), g.rowptr.data_ptr(), g.col.data_ptr(),
          s["W"].data_ptr(), s["a_s"].data_ptr(), s["a_d"].data_ptr(), bias.data_ptr(), H, C, 0.2, 0.0, 0,
          plan.cstruct(), out.data_ptr(), st.data_ptr(), stats.data_ptr(), ws.data_ptr(), ws.numel(), _lib.stream_handle(DEV))
M = g.num_messages
bws = torch.zeros(lib.gfd_gat_bwd_workspace_size(N, M, F, H, C, plan.num_hubs, plan.num_chunks, splan.num_chunks), dtype=torch.uint8, device=DEV)
gw = torch.empty((512, F), device=DEV); gas = torch.empty(512, device=DEV); gad = torch.empty(512, device=DEV); gb = torch.empty(64, device=DEV)
gd = gout.to(DEV)
_lib.call("gfd_gat_bwd", x.data_ptr(), 0, N, F, x.stride(0), g.rowptr.data_ptr(), g.col.data_ptr(), plan.cstruct(),
          csc.colptr.data_ptr(), csc.dst.data_ptr(), csc.eid.data_ptr(), splan.cstruct(), M,
          s["W"].data_ptr(), s["a_s"].data_ptr(), s["a_d"].data_ptr(), H, C, 0.2, 0.0, 0, st.data_ptr(), stats.data_ptr(),
          gd.data_ptr(), None, gw.data_ptr(), gas.data_ptr(), gad.data_ptr(), gb.data_ptr(), bws.data_ptr(), bws.numel(),
          _lib.stream_handle(DEV))
torch.cuda.synchronize()
def al(o): return (o + 255) // 256 * 256
Fu = (F + 15) // 16 * 16; NT = Fu // 16
o = 0; offs = {}
for name, nb in (("whdr", 64), ("amax", 64), ("bhi", 16 * H * 2 * NT * 64), ("blo", 16 * H * 2 * NT * 64),
                 ("dpre", 4 * M * 8), ("alpha", 4 * M * 8), ("dt", 4 * N * 8)):
    o = al(o); offs[name] = o; o += nb
def wsf(name, n): return bws[offs[name]:offs[name] + 4 * n].view(torch.float32)
dpre = wsf("dpre", M * 8).view(M, 8); alpha = wsf("alpha", M * 8).view(M, 8); dt = wsf("dt", N * 8).view(N, 8)
W = s["W"].double().cpu(); a_s = s["a_s"].double().cpu().view(H, C); a_d = s["a_d"].double().cpu().view(H, C)
rp = g.rowptr.long().cpu(); col = g.col.long().cpu(); cp = csc.colptr.long().cpu()
cdst = csc.dst.long().cpu(); ceid = csc.eid.long().cpu()
hub_rank = plan.hub_rank.cpu() if plan.num_hubs else None
order = plan.row_order.long().cpu(); inv = torch.empty_like(order); inv[order] = torch.arange(N)
a, b = plan.classes()
def hrow(j): return (x[j].double().cpu() @ W.t()).view(H, C)
for j in nodes:
    print(f"=== node {j}: in {int(rp[j+1]-rp[j])} out {int(cp[j+1]-cp[j])}")
    for p in range(int(cp[j]), int(cp[j + 1])):
        i, e = int(cdst[p]), int(ceid[p])
        js = col[rp[i]:rp[i + 1]]
        hj = torch.stack([hrow(int(v)) for v in js])          # [k, H, C]
        hi = hrow(i)
        ssrc = (hj * a_s).sum(-1); tdst = (hi * a_d).sum(-1)
        pre = ssrc + tdst
        lg = Fn.leaky_relu(pre, 0.2)
        mx = lg.max(0).values; ex = (lg - mx).exp(); sm = ex.sum(0)
        alp = ex / (sm + 1e-16)
        gi = gout[i].double()
        dA = (hj * gi.view(1, 1, C)).sum(-1) / H
        adot = (alp * dA).sum(0)
        dp = alp * (dA - adot) * torch.where(pre > 0, 1.0, 0.2)
        k = e - int(rp[i])
        slot = int(inv[i]); cls = "general" if slot < a else ("light" if slot < b else "lone")
        hub = bool(hub_rank[i] >= 0) if hub_rank is not None else False
        print(f"  msg e={e} -> dst {i} (deg {len(js)}, slot {slot} {cls}, hub {hub}, pos {k})")
        print("    stats max gpu", [round(v, 5) for v in stats[i, :8].tolist()], "ref", [round(v, 5) for v in mx.tolist()])
        print("    stats sum gpu", [round(v, 5) for v in stats[i, 8:].tolist()], "ref", [round(v, 5) for v in sm.tolist()])
        print("    alpha gpu", [round(v, 5) for v in alpha[e].tolist()], "ref", [round(v, 5) for v in alp[k].tolist()])
        print("    dpre  gpu", [round(v, 6) for v in dpre[e].tolist()], "ref", [round(v, 6) for v in dp[k].tolist()])
        print("    dt    gpu", [round(v, 6) for v in dt[i].tolist()], "ref", [round(v, 6) for v in dp.sum(0).tolist()])
