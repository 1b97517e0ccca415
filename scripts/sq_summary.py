#!/usr/bin/env python3
"""Per-kernel averages of the SQ counter passes written by scripts/gpu_sq2.sh.
usage: sq_summary.py gpurun_out/<TAG>_1 gpurun_out/<TAG>_2 [kernel-prefix]"""
import collections, csv, glob, os, sys

def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(path)):
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
            acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc

pref = sys.argv[-1] if not os.path.isdir(sys.argv[-1]) else "k_"
tot = collections.defaultdict(dict)
for d in [a for a in sys.argv[1:] if os.path.isdir(a)]:
    for k, cs in load(d).items():
        for c, v in cs.items():
            tot[k][c] = sum(v) / len(v)
for k in sorted(tot):
    if not k.startswith(pref):
        continue
    print(k)
    for c in sorted(tot[k]):
        print(f"   {c:28s} {tot[k][c]:16.4g}")
