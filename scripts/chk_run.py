#!/usr/bin/env python3
"""Run sharded / single forwards through the bounds-checked build (GFD_LIB_PATH ->
libgfd_chk.so) and print the first out-of-range index k_stream saw, per call."""
import ctypes, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd"), os.path.join(REPO, "tests")]
os.environ.setdefault("GFD_LIB_PATH", os.path.join(REPO, "gnn-fraud-detection_amd", "gfd", "libgfd_chk.so"))
import torch
from gfd import _lib, dist as gdist, graph as ggraph, synth
from oracle import gatconv_ref as ref
lib = _lib.load()
buf = (ctypes.c_longlong * 4)()
def chk(tag):
    torch.cuda.synchronize()
    if not hasattr(lib, "gfd_debug_chk"):
        print(f"{tag}: ok (unchecked build)", flush=True)
        return
    lib.gfd_debug_chk(buf)
    print(f"{tag}: site={buf[0]} value={buf[1]} limit={buf[2]} block*1000+wave={buf[3]}", flush=True)
dev = torch.device("cuda", 0)
H, C = 8, 64
for (N, E, F, world) in [(20000, 160000, 166, 2), (20000, 160000, 166, 1), (3000, 3450, 166, 1),
                         (20000, 160000, 128, 2), (20000, 160000, 100, 1), (20000, 160000, 64, 3),
                         (20000, 160000, 17, 1)]:
    g = torch.Generator().manual_seed(11)
    ei = torch.from_numpy(synth.power_law(N, E, gamma=2.1, seed=11))
    x = torch.randn(N, F, generator=g)
    W = ref.glorot_(torch.empty(H * C, F), g)
    a_s = ref.glorot_(torch.empty(1, H, C), g)
    a_d = ref.glorot_(torch.empty(1, H, C), g)
    b = torch.randn(C, generator=g) * 0.1
    gr = ggraph.csr_from_coo(ei.to(dev), N)
    xd = x.to(dev)
    packed = gdist.pack_weights(W.to(dev), a_s.to(dev), a_d.to(dev))
    specs = [gdist.ShardSpec(gr.rowptr, r, world) for r in range(world)]
    st = torch.cat([gdist.shard_logits(xd, packed, s) for s in specs])
    outs = []
    for s in specs:
        outs.append(gdist.shard_aggregate(xd, gr, st, packed, b.to(dev), s))
        chk(f"N={N} world={world} rank={s.rank if hasattr(s, 'rank') else '?'}")
    out = torch.cat(outs).cpu()
    exp = ref.gatconv_forward(x, ei, W, a_s, a_d, b, heads=H)
    print("   max err", (out - exp).abs().max().item(), flush=True)
