#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV: per kernel (short name) the call
count, mean / median duration, and the resources of its dispatches."""
import csv
import re
import statistics
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = n.split("(")[0]
    n = n.replace("gfd::fwd::", "")
    return n[:110]


def main(path: str, top: int = 14):
    rows = list(csv.DictReader(open(path)))
    by = defaultdict(list)
    res = {}
    for r in rows:
        k = short(r["Kernel_Name"])
        by[k].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
        res[k] = (r.get("VGPR_Count"), r.get("Accum_VGPR_Count"), r.get("SGPR_Count"),
                  r.get("LDS_Block_Size"), r.get("Scratch_Size"), r.get("Grid_Size_X"),
                  r.get("Workgroup_Size_X"))
    tot = sum(sum(v) for v in by.values())
    items = sorted(by.items(), key=lambda kv: -sum(kv[1]))[:top]
    print(f"{'kernel':110s} {'n':>4} {'mean_ms':>8} {'med_ms':>8} {'%':>6}  vgpr/agpr/sgpr lds scratch grid wg")
    for k, v in items:
        print(f"{k:110s} {len(v):4d} {statistics.mean(v):8.3f} {statistics.median(v):8.3f} "
              f"{100 * sum(v) / tot:6.2f}  {'/'.join(str(x) for x in res[k][:3])} {res[k][3]} "
              f"{res[k][4]} {res[k][5]} {res[k][6]}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 14)
