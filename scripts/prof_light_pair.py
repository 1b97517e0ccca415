"""Phase split of the paired-phase light kernel (diagnostic): runs the bench
layer with the -DGFD_LP_PROF build (GFD_LIB_PATH) and prints, per wave group,
cycles per step of each kind and where they go.

    cd gnn-fraud-detection_amd && GFD_BUILD_VARIANT=lpprof GFD_EXTRA_FLAGS=-DGFD_LP_PROF python -m gfd.build
    GFD_LIB_PATH=$PWD/gnn-fraud-detection_amd/gfd/libgfd_lpprof.so python scripts/prof_light_pair.py [--config c5]
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
    rd = lib.gfd_lprof_read
    rd.argtypes = [ct.c_void_p, ct.c_int]
    buf = (ct.c_ulonglong * 32)()
    for _ in range(2):
        layer.step()
    torch.cuda.synchronize()
    rd(buf, 1)
    for _ in range(5):
        layer.step()
    torch.cuda.synchronize()
    rd(buf, 0)
    for g in (0, 1):
        v = [buf[16 * g + i] for i in range(7)]
        w = [buf[16 * g + 8 + i] for i in range(4)]
        ns, nm = max(v[5], 1), max(v[6], 1)
        print(f"{'C5' if c5 else 'C4'} group {g}: aggregation step {v[0] / ns:.0f} cyc "
              f"(rows wait {v[1] / ns:.0f}), barrier after it {v[3] / ns:.0f}; "
              f"MFMA step {v[2] / nm:.0f} cyc, barrier after it {v[4] / nm:.0f}  "
              f"[{v[5]} / {v[6]} wave-steps]")
        print("   aggregation step: " + ", ".join(
            f"{n} {x / ns:.0f}" for n, x in zip(("softmax", "aggregate (2 passes)", "rows issue",
                                                 "logits + records"), w)))


if __name__ == "__main__":
    main()
