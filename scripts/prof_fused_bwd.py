"""Phase split of the fused backward source pass (diagnostic): the C4 layer
forward + backward with GFD_BWD_FUSED=1 through the -DGFD_FPROF build of
libgfd (GFD_LIB_PATH); prints the share of k_src_gw's wave cycles per phase
of its tile loop and cycles per tile.

    cd gnn-fraud-detection_amd && GFD_BUILD_VARIANT=fprof GFD_EXTRA_FLAGS=-DGFD_FPROF python -m gfd.build
    GFD_BWD_FUSED=1 GFD_LIB_PATH=$PWD/gnn-fraud-detection_amd/gfd/libgfd_fprof.so python scripts/prof_fused_bwd.py
"""
import ctypes as ct
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from gfd import _lib  # noqa: E402
from gfd.nn import gat_conv  # noqa: E402


def main():
    os.environ["GFD_BWD_FUSED"] = "1"
    dev = torch.device("cuda:0")
    s = bench.setup(dev, 10_000_000, 50_000_000, 166)
    W = s["W"].clone().requires_grad_(True)
    a_s = s["a_s"].clone().requires_grad_(True)
    a_d = s["a_d"].clone().requires_grad_(True)
    b = s["bias"].clone().requires_grad_(True)
    g = s["graph"]
    grad = torch.randn((g.num_nodes, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(4))
    rd = _lib.load().gfd_fprof_read
    rd.argtypes = [ct.c_void_p, ct.c_int]
    buf = (ct.c_ulonglong * 10)()

    def step():
        gat_conv(s["x"], g, W, a_s, a_d, b, training=True).backward(grad)

    step()
    torch.cuda.synchronize()
    rd(buf, 1)
    steps = 3
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    rd(buf, 0)
    names = {0: "MFMA(t-1)", 1: "prefix + loads issue", 2: "walk (consume, flush)",
             3: "hub rows + barrier A", 6: "next chunk's data issue", 7: "x tile -> B image",
             4: "merge", 5: "column pass + barrier B"}
    tot = sum(buf[i] for i in range(8))
    tiles = buf[8]   # wave-tiles (every wave adds its block's T)
    for i, n in names.items():
        print(f"{n:30s} {100.0 * buf[i] / max(tot, 1):6.1f} %  {buf[i] / max(tiles, 1):9.0f} cyc/tile")
    print(f"{'total':30s} {'':8s} {tot / max(tiles, 1):9.0f} cyc/tile  ({buf[8] // 8 // steps} block-tiles per pass)")


if __name__ == "__main__":
    main()
