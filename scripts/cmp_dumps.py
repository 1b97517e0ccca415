"""Compare two scripts/dump_fwd.py dumps (gpurun_out/<a>.npz, <b>.npz): max |diff| and
the count of differing elements per array (bit-identity check of kernel variants)."""
import sys

import numpy as np

a = np.load(f"gpurun_out/{sys.argv[1]}.npz")
b = np.load(f"gpurun_out/{sys.argv[2]}.npz")
for k in a.files:
    x, y = a[k], b[k]
    if x.dtype.kind == "f":
        d = np.abs(x.astype(np.float64) - y)
        print(f"{k:12s} max|diff| {d.max():.3e} differing {(x != y).sum()} of {x.size}")
    else:
        print(f"{k:12s} equal {np.array_equal(x, y)}")
