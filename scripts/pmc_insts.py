#!/usr/bin/env python3
"""Per-kernel instruction mix from the rocprofv3 --pmc passes of
scripts/gpu_pmc_all.sh (P1: wave states, P2: SQ_INSTS_*), per dispatch and
per unit of work (e.g. light destinations):

    python3 scripts/pmc_insts.py DIR... --per 'k_stream<XF32, 3, 21, 8, true, true>=6203351'

SQ_WAVE_CYCLES / SQ_WAIT_* count quad-cycles (MI355X_MICROARCH.md); the
instruction counters count wave-instructions."""
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_table import load  # noqa: E402

KEYS = ["SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS", "SQ_INSTS_VMEM_RD",
        "SQ_INSTS_SMEM", "SQ_WAIT_INST_ANY", "SQ_WAIT_ANY", "SQ_ACTIVE_INST_ANY",
        "SQ_WAVE_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES"]


def main(argv):
    per_arg = {}
    dirs = []
    i = 0
    while i < len(argv):
        if argv[i] == "--per":
            k, v = argv[i + 1].rsplit("=", 1)
            per_arg[k] = float(v)
            i += 2
        else:
            dirs.append(argv[i])
            i += 1
    per, calls = load(dirs)
    for k in sorted(per, key=lambda k: -per[k].get("SQ_WAVE_CYCLES", 0)):
        c = per[k]
        if "SQ_INSTS_VALU" not in c:
            continue
        n = max(calls[k], 1)
        units = per_arg.get(k)
        vals = {key: c.get(key, 0.0) / n for key in KEYS}
        line = f"{k[:60]:60s} x{n} " + " ".join(f"{key[3:]}={v:.4g}" for key, v in vals.items())
        print(line)
        if units:
            print(f"    per unit ({units:.0f}): " +
                  " ".join(f"{key[3:]}={v / units:.2f}" for key, v in vals.items()))


if __name__ == "__main__":
    main(sys.argv[1:])
