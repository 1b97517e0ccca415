#!/usr/bin/env python3
"""Fold the rocprofv3 --pmc passes of scripts/gpu_pmc.sh into profiles/pmc_summary.json.

Per kernel (averaged over its dispatches): FETCH_SIZE and WRITE_SIZE (KiB in the
CSV), converted to bytes.  On gfx950 FETCH_SIZE tallies 128-B requests at 64 B
(MI355X_MICROARCH.md § HBM), so ``fetch_bytes`` = 2 x the raw figure; WRITE_SIZE
is exact.  ``hbm_bytes_per_launch`` = fetch_bytes + write_bytes of the tile
kernel, keyed by the bench workload, which bench.py reports as roofline.traffic.

usage: pmc_summary.py <gpurun_out dir> N E F world [tag]
"""
import csv
import collections
import json
import os
import sys


def per_kernel(path):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        acc[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def main():
    d, N, E, F, world = sys.argv[1], *map(int, sys.argv[2:6])
    tag = sys.argv[6] if len(sys.argv) > 6 else ""
    fetch = per_kernel(os.path.join(d, "pmc_FETCH_SIZE", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(d, "pmc_WRITE_SIZE", "run_counter_collection.csv"))
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out_path = os.path.join(repo, "profiles", "pmc_summary.json")
    try:
        summary = json.load(open(out_path))
    except (OSError, ValueError):
        summary = {}
    kernels = {}
    for k in sorted(set(fetch) & set(write)):
        if not k.startswith("k_"):
            continue
        fb = 2 * fetch[k] * 1024
        wb = write[k] * 1024
        kernels[k] = {"fetch_size_kib_raw": fetch[k], "fetch_bytes": fb, "write_bytes": wb,
                      "hbm_bytes_per_launch": fb + wb}
    # the tile stage is k_split + the k_stream launches (general + light tiles), or k_fused
    tile = sorted(k for k in kernels if k.startswith(("k_stream", "k_fused", "k_persist", "k_split")))
    entry = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (two passes) {tag}",
             "fetch_correction": "x2 (gfx950 FETCH_SIZE counts 128-B requests at 64 B)",
             "kernels": kernels}
    if tile:
        entry["tile_kernel"] = " + ".join(tile)
        entry["hbm_bytes_per_launch"] = sum(kernels[k]["hbm_bytes_per_launch"] for k in tile)
    summary[f"tile:N={N}:E={E}:F={F}:world={world}"] = entry
    json.dump(summary, open(out_path, "w"), indent=1, sort_keys=True)
    for k, v in kernels.items():
        print(f"{k:28s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
