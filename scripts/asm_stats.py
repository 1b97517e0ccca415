"""Instruction mix of one kernel in a hipcc -S listing, per basic block.

    python scripts/asm_stats.py /tmp/asm/fwd.s 'k_streamILi3ELi21ELi8ELb1E' [--blocks]

Classes: mfma, valu (v_*), salu (s_* except waits/branches), lds (ds_*), vmem
(global_/buffer_), smem (s_load/s_buffer_load), wait (s_waitcnt), branch.
"""
import re
import sys
from collections import Counter, OrderedDict


def classify(op):
    if op.startswith("v_mfma"):
        return "mfma"
    if op.startswith("v_"):
        return "valu"
    if op.startswith("ds_"):
        return "lds"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "vmem"
    if op.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if op.startswith("s_waitcnt"):
        return "wait"
    if op.startswith(("s_cbranch", "s_branch", "s_setpc", "s_endpgm")):
        return "branch"
    if op.startswith("s_"):
        return "salu"
    return "other"


def main():
    path, pat = sys.argv[1], sys.argv[2]
    lines = open(path).read().splitlines()
    start = next(i for i, l in enumerate(lines) if re.match(r"^_Z\S*" + pat + r"\S*:", l))
    blocks = OrderedDict()
    cur = "entry"
    blocks[cur] = Counter()
    for l in lines[start + 1:]:
        if l.startswith(".Lfunc_end"):
            break
        m = re.match(r"^(\.LBB\S+):", l)
        if m:
            cur = m.group(1)
            blocks[cur] = Counter()
            continue
        t = l.strip()
        if not t or t.startswith((";", ".")):
            continue
        op = t.split()[0]
        blocks[cur][classify(op)] += 1
        blocks[cur]["_ops"] += 1
    total = Counter()
    for c in blocks.values():
        total.update(c)
    keys = ["mfma", "valu", "salu", "lds", "vmem", "smem", "wait", "branch"]
    print("total", " ".join(f"{k}={total[k]}" for k in keys))
    if "--blocks" in sys.argv:
        for name, c in blocks.items():
            print(f"{name:12s}", " ".join(f"{k}={c[k]}" for k in keys if c[k]))


if __name__ == "__main__":
    main()
