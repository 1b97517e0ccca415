#!/usr/bin/env python3
"""Fold the rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of scripts/gpu_pmc.sh
into profiles/pmc_summary.json, per bench stage.

Per kernel (averaged over its dispatches): FETCH_SIZE and WRITE_SIZE (KiB in the
CSV), converted to bytes.  On gfx950 FETCH_SIZE tallies 128-B requests at 64 B
(MI355X_MICROARCH.md § HBM), so ``fetch_bytes`` = 2 x the raw figure; WRITE_SIZE
is exact.  Each bench stage (bench.py ``kernels``) gets ``hbm_bytes_per_launch``
= the sum over its kernels, keyed ``{config}:{stage}:N=..:E=..:F=..:world=..``;
bench.py reports the dominant stage's figure as ``roofline.traffic``.

usage: GFD_TREE=<git hash> pmc_summary.py <fetch pass dir> <write pass dir> CONFIG N E F WORLD [tag]
"""
import collections
import csv
import glob
import json
import os
import sys


def per_kernel(d):
    paths = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not paths:
        raise SystemExit(f"no counter_collection.csv under {d}")
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(paths[0])):
        name = r["Kernel_Name"]
        short = name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        short = short.replace("gfd::fwd::", "")
        acc[short].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in acc.items()}


def stage_of(k):
    if k.startswith("k_stream<"):
        # k_stream<XT, KF, KHM, LO, EXACT, LIGHT, EPI>; LIGHT 0 general, 1 light,
        # 2 short light (round 6; "true" / "false" before)
        args = [a.strip() for a in k[k.index("<") + 1:k.rindex(">")].split(",")]
        return "light" if args[5] in ("true", "1", "2") else "general"
    if k.startswith(("k_hub_partial", "k_hub_fin")):
        return "hubs"
    if k.startswith(("k_logits_lone", "k_wmax", "k_pack_")):
        return "pack+logits+lone"
    if k.startswith("k_lone"):
        return "lone"
    return None


def main():
    fd, wd, config = sys.argv[1], sys.argv[2], sys.argv[3]
    N, E, F, world = map(int, sys.argv[4:8])
    tag = sys.argv[8] if len(sys.argv) > 8 else ""
    fetch, write = per_kernel(fd), per_kernel(wd)
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
    stages = collections.defaultdict(list)
    for k in kernels:
        s = stage_of(k)
        if s:
            stages[s].append(k)
    for s, ks in stages.items():
        summary[f"{config}:{s}:N={N}:E={E}:F={F}:world={world}"] = {
            "source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE --kernel-trace (two passes) {tag}",
            # the git tree the passes ran on (GFD_TREE: set by the caller, the
            # GPU box's snapshot has no .git)
            "tree": os.environ.get("GFD_TREE", "unknown"),
            "fetch_correction": "x2 (gfx950 FETCH_SIZE counts 128-B requests at 64 B)",
            "kernels": {k: kernels[k] for k in sorted(ks)},
            "hbm_bytes_per_launch": sum(kernels[k]["hbm_bytes_per_launch"] for k in ks),
        }
    json.dump(summary, open(out_path, "w"), indent=1, sort_keys=True)
    for k, v in kernels.items():
        print(f"{k:60s} fetch {v['fetch_bytes'] / 1e9:8.3f} GB  write {v['write_bytes'] / 1e9:8.3f} GB")
    for s, ks in stages.items():
        print(f"stage {s:18s} {sum(kernels[k]['hbm_bytes_per_launch'] for k in ks) / 1e9:8.3f} GB")


if __name__ == "__main__":
    main()
