"""Random-row gather rate vs. footprint (diagnostic): is a gather of x rows
limited by bytes, or by the row rate of a large x (TLB / DRAM page locality)?
Uses scripts/libgather_probe.so (hipcc -shared scripts/gather_probe.hip).

    python scripts/gather_probe.py
"""
import ctypes as ct
import os

import torch

lib = ct.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "libgather_probe.so"))
lib.probe_gather.argtypes = [ct.c_void_p, ct.c_int, ct.c_int64, ct.c_int, ct.c_void_p, ct.c_int64,
                             ct.c_void_p, ct.c_int, ct.c_void_p]
dev = "cuda"
torch.manual_seed(0)
F, LD = 166, 168
R = 48_000_000
big = torch.randn(10_000_000, LD, device=dev)
bigh = big.to(torch.bfloat16)
cus = torch.cuda.get_device_properties(0).multi_processor_count
out = torch.empty(cus * 8 * 4 * 256, device=dev)
stream = torch.cuda.current_stream().cuda_stream


def rate(x, rows, blocks_per_cu, tag, stride=1):
    idx = (torch.randint(0, rows, (R,), device=dev, dtype=torch.int32) * stride).contiguous()
    nb = cus * blocks_per_cu
    bf = 1 if x.dtype == torch.bfloat16 else 0
    run = lambda: lib.probe_gather(x.data_ptr(), bf, LD, F, idx.data_ptr(), R // 8, out.data_ptr(),  # noqa: E731
                                   nb, stream)
    run()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(True), torch.cuda.Event(True)
    e0.record()
    for _ in range(5):
        run()
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 5
    gb = R * F * x.element_size() / 1e9
    print(f"{tag:28s} blocks/CU {blocks_per_cu}  footprint {rows * stride * LD * x.element_size() / 1e9:6.2f} GB"
          f"  {ms:7.3f} ms  {R / ms / 1e6:6.2f} G rows/s  {gb / ms:6.2f} TB/s", flush=True)


for occ in (4, 8):
    for rows in (10_000_000, 1_000_000, 100_000):
        rate(big, rows, occ, f"fp32 rows<{rows}")
    rate(big, 100_000, occ, "fp32 100k rows, stride 100", stride=100)
for rows in (10_000_000, 100_000):
    rate(bigh, rows, 8, f"bf16 rows<{rows}")
