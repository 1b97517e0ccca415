#!/usr/bin/env python3
"""Per-kernel co-execution table from scripts/gpu_coexec.sh's passes.

SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_* count quad-cycles, SQ_VALU_MFMA_BUSY
and SQ_VALU_MFMA_COEXEC count cycles (MI355X_MICROARCH.md).  Printed per
dispatch: instruction counts, the wave-state split, MFMA busy cycles and the
fraction of them during which vector instructions executed too."""
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from pmc_table import load  # noqa: E402


def main(dirs):
    per, calls = load(dirs)
    for k in sorted(per, key=lambda k: -per[k].get("SQ_WAVE_CYCLES", 0)):
        c = per[k]
        if "SQ_WAVE_CYCLES" not in c:
            continue
        n = max(calls[k], 1)
        wc = c["SQ_WAVE_CYCLES"]
        busy = c.get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
        co = c.get("SQ_VALU_MFMA_COEXEC_CYCLES", 0.0)
        ins = " ".join(f"{key[9:]}={c.get(key, 0) / n:.4g}" for key in
                       ("SQ_INSTS_VALU", "SQ_INSTS_MFMA", "SQ_INSTS_SALU", "SQ_INSTS_LDS",
                        "SQ_INSTS_VMEM_RD") if key in c)
        print(f"{k[:64]:64s} x{n} {ins}")
        print(f"{'':64s}   wave_cyc {wc / n:.4g} (quad) wait_any {c.get('SQ_WAIT_ANY', 0) / wc:.3f} "
              f"wait_inst {c.get('SQ_WAIT_INST_ANY', 0) / wc:.3f} active {c.get('SQ_ACTIVE_INST_ANY', 0) / wc:.3f} "
              f"mfma_busy {busy / n:.4g} coexec {co / n:.4g} coexec/busy {co / busy if busy else 0:.3f}")


if __name__ == "__main__":
    main(sys.argv[1:])
