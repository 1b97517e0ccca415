"""Phase split of the tile kernels (diagnostic): runs the bench layer with the
-DGFD_PROF build of libgfd (GFD_LIB_PATH) and prints, per class, the share of
wave cycles in each phase of the k_stream tile loop and cycles per tile.

    cd gnn-fraud-detection_amd && GFD_BUILD_VARIANT=prof GFD_EXTRA_FLAGS=-DGFD_PROF python -m gfd.build
    GFD_LIB_PATH=$PWD/gnn-fraud-detection_amd/gfd/libgfd_prof.so python scripts/prof_phases.py [--config c5]
"""
import ctypes as ct
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "gnn-fraud-detection_amd")]
import torch  # noqa: E402

import bench  # noqa: E402
from gfd import _lib  # noqa: E402


def main():
    c5 = "--config" in sys.argv and sys.argv[sys.argv.index("--config") + 1] == "c5"
    dev = torch.device("cuda:0")
    N, E, dt = (50_000_000, 500_000_000, torch.bfloat16) if c5 else (10_000_000, 50_000_000, torch.float32)
    s = bench.setup(dev, N, E, 166, 2.1, dt)
    layer = bench.Layer(s, dev, 1)
    lib = _lib.load()
    rd = lib.gfd_prof_read
    rd.argtypes = [ct.c_void_p, ct.c_int]
    buf = (ct.c_ulonglong * 18)()
    for _ in range(2):
        layer.step()
    torch.cuda.synchronize()
    rd(buf, 1)
    steps = 5
    for _ in range(steps):
        layer.step()
    torch.cuda.synchronize()
    rd(buf, 0)
    names = ("MFMA + next-tile issue", "barrier 1", "aggregation", "barrier 2")
    for cls, k in (("general", 0), ("light", 1), ("short light", 2)):
        v = [buf[6 * k + i] for i in range(6)]
        tot = sum(v[:4])
        tiles = v[4] / steps
        waves_per_tile = 8
        print(f"{'C5' if c5 else 'C4'} {cls}: {tiles:.0f} tiles/step, "
              f"{tot / steps / max(tiles, 1) / waves_per_tile:.0f} cycles per tile (per wave)")
        for n, x in zip(names, v[:4]):
            print(f"   {n:24s} {100.0 * x / max(tot, 1):5.1f} %")
        print(f"   {'(of aggregation: rows)':24s} {100.0 * v[5] / max(tot, 1):5.1f} %")


if __name__ == "__main__":
    main()
