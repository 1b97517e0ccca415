"""Locate backward errors per node: run gfd_gat_bwd directly with a caller-held
workspace, read its dh' rows ([N, 528] = dh | ds | dt) and compare dh with the
fp64 chunked oracle's dL/dh per node; report the worst nodes and their degrees."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import torch
import bench
from gfd import _lib
from gfd.nn import gat_conv
from oracle import gatconv_grads_chunked

N = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
DEV = torch.device("cuda", 0)
s = bench.setup(DEV, N, 5 * N, 166)
g = s["graph"]
csc = g.csc()
plan, splan = g.plan(), csc.plan
F, H, C = 166, 8, 64
gen = torch.Generator().manual_seed(6)
bias = (torch.randn(64, generator=gen) * 0.1).to(DEV)
gout = torch.randn((N, 64), generator=gen)
x = s["x"]
# forward with stats
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
o = 0
offs = {}
# mirrors bwd_layout() in gfd_gat_bwd.hip
for name, nb in (("whdr", 64), ("amax", 4 * (528 + 256)), ("erow", 4 * N),
                 ("bhi", 16 * H * 2 * NT * 64), ("blo", 16 * H * 2 * NT * 64),
                 ("rec", 4 * M * 16), ("dt", 4 * N * 8),
                 ("uhub", 4 * plan.num_hubs * H * Fu), ("cpart", 4 * plan.num_chunks * 8), ("hadot", 4 * plan.num_hubs * 8),
                 ("spart", 4 * splan.num_chunks * 520), ("dh", 4 * N * 528)):
    o = al(o); offs[name] = o; o += nb
dhp = bws[offs["dh"]:offs["dh"] + 4 * N * 528].view(torch.float32).view(N, 528).cpu().double()
ref = gatconv_grads_chunked(x.cpu(), g.rowptr.cpu(), g.col.cpu(), s["W"].cpu(), s["a_s"].cpu(), s["a_d"].cpu(),
                            bias.cpu(), gout, dtype=torch.float64)
dh_ref = ref["dh"]
err = (dhp[:, :512] - dh_ref).abs()
print("grad_W err vs oracle:", (gw.cpu().double() - ref["weight"]).abs().max().item())
rowerr = err.max(1).values
top = torch.topk(rowerr, 20)
rp = g.rowptr.long().cpu(); cp = csc.colptr.long().cpu()
indeg = rp[1:] - rp[:-1]; outdeg = cp[1:] - cp[:-1]
hubdst = plan.hub_rank.cpu()[:N] >= 0 if plan.num_hubs else torch.zeros(N, dtype=torch.bool)
hubsrc = splan.hub_rank.cpu()[:N] >= 0 if splan.num_hubs else torch.zeros(N, dtype=torch.bool)
print("amax", bws[offs["amax"]:offs["amax"] + 8].view(torch.float32).tolist())
print("max |dh| ref", dh_ref.abs().max().item())
for v, j in zip(top.values.tolist(), top.indices.tolist()):
    e = err[j].view(8, 64).max(1).values
    print(f"node {j}: err {v:.4g} |dh| {dh_ref[j].abs().max().item():.4g} in {indeg[j].item()} out {outdeg[j].item()} "
          f"hubdst {bool(hubdst[j])} hubsrc {bool(hubsrc[j])} per-head {[round(t, 4) for t in e.tolist()]}")
bad = rowerr > 1e-3 * dh_ref.abs().max()
print("nodes with err > 1e-3 max:", int(bad.sum()), "of which hub src", int((bad & hubsrc).sum()), "hub dst", int((bad & hubdst).sum()))
