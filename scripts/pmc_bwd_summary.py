#!/usr/bin/env python3
"""Fold the backward PMC passes of scripts/gpu_bwd_pmc.sh (FETCH_SIZE,
WRITE_SIZE over bench.py --legs c4bwd) into profiles/pmc_summary.json as
"c4:backward:N=<N>:world=1": per backward kernel the HBM bytes per launch
(FETCH_SIZE doubled: MI355X_MICROARCH.md §HBM, calibrated for this path's
access widths in profiles/r3c_fetch_probe.txt) and their sum per backward pass.
Entries are stamped with the tree they came from (GFD_TREE, e.g. the short
commit hash of the tree the passes ran on).

    GFD_TREE=$(git rev-parse --short HEAD) python scripts/pmc_bwd_summary.py \
        gpurun_out/r3cbwd_fetch gpurun_out/r3cbwd_write 10000000 r3cbwd
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(__file__))
from pmc_table import load  # noqa: E402

BWD = ("k_bwd_", "k_gw", "k_xmax", "k_colsum64", "k_reduce_", "k_att_grad", "k_sum8", "k_gx",
       "k_gemm")


def main(fetch_dir, write_dir, n, tag):
    per, calls = load([fetch_dir, write_dir])
    kern = {}
    for k, c in per.items():
        if not k.startswith(BWD):
            continue
        ncall = max(calls[k], 1)
        # launches per backward pass: k_sum8 runs twice per pass
        per_pass = 2 if k.startswith("k_sum8") else 1
        f = 2 * c.get("FETCH_SIZE", 0.0) * 1024 / ncall
        w = c.get("WRITE_SIZE", 0.0) * 1024 / ncall
        kern[k] = {"fetch_bytes": f, "write_bytes": w, "hbm_bytes_per_launch": f + w,
                   "launches_per_pass": per_pass}
    total = sum(v["hbm_bytes_per_launch"] * v["launches_per_pass"] for v in kern.values())
    path = os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_summary.json")
    try:
        with open(path) as fh:
            summ = json.load(fh)
    except (OSError, ValueError):
        summ = {}
    summ[f"c4:backward:N={n}:world=1"] = {
        "hbm_bytes_per_pass": total, "kernels": kern,
        "fetch_correction": "x2 (gfx950 FETCH_SIZE counts half; profiles/r3c_fetch_probe.txt)",
        "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (two passes) {tag}, "
                  "bench.py --legs c4bwd",
        "tree": os.environ.get("GFD_TREE", "unknown")}
    with open(path, "w") as fh:
        json.dump(summ, fh, indent=1, sort_keys=True)
    print(f"backward HBM bytes per pass: {total / 1e9:.2f} GB over {len(kern)} kernels")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4])
