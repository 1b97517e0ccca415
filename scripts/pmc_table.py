#!/usr/bin/env python3
"""Per-kernel PMC table from rocprofv3 --pmc counter_collection CSVs (one or
more passes): counters summed over a kernel's dispatches, divided by the
dispatch count.  FETCH_SIZE is doubled (MI355X_MICROARCH.md: gfx950 reports
half the bytes of a wide streaming read) and reported with WRITE_SIZE in
bytes (the CSV values are KB)."""
import csv
import glob
import sys
from collections import defaultdict

sys.path.insert(0, __import__("os").path.dirname(__file__))
from kstats import short  # noqa: E402


def load(dirs):
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for d in dirs:
        for path in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(path)):
                k = short(r["Kernel_Name"])
                disp[(k, d)].add(r["Dispatch_Id"])
                per[k][r["Counter_Name"]] += float(r["Counter_Value"])
    calls = defaultdict(int)
    for (k, d), s in disp.items():
        calls[k] = max(calls[k], len(s))
    return per, calls


def main(dirs, names=None):
    per, calls = load(dirs)
    for k in sorted(per, key=lambda k: -per[k].get("SQ_WAVE_CYCLES", per[k].get("FETCH_SIZE", 0))):
        if names and not any(n in k for n in names):
            continue
        c = per[k]
        n = max(calls[k], 1)
        out = []
        if "FETCH_SIZE" in c:
            out.append(f"fetch {2 * c['FETCH_SIZE'] * 1024 / n / 1e9:.3f} GB")
        if "WRITE_SIZE" in c:
            out.append(f"write {c['WRITE_SIZE'] * 1024 / n / 1e9:.3f} GB")
        if "SQ_WAVE_CYCLES" in c:
            wc = c["SQ_WAVE_CYCLES"]
            out.append(f"wave_cyc {wc / n:.3e} wait_any {c.get('SQ_WAIT_ANY', 0) / wc:.2f} "
                       f"wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.2f} "
                       f"active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.2f} "
                       f"valu/vmem {c.get('SQ_ACTIVE_INST_VALU', 0) / max(c.get('SQ_ACTIVE_INST_VMEM', 1), 1):.1f} "
                       f"busy {c.get('SQ_BUSY_CYCLES', 0) / n:.3e}")
        print(f"{k[:60]:60s} x{n} " + " | ".join(out))


if __name__ == "__main__":
    args = sys.argv[1:]
    names = None
    if "--only" in args:
        i = args.index("--only")
        names = args[i + 1].split(",")
        args = args[:i] + args[i + 2:]
    main(args, names)
