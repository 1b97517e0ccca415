#!/bin/bash
# Round-5 GPU check: selected tests, then bench lines (A/B pairs of bench
# argument sets, each its own process).
# usage: scripts/gpu_r5.sh TAG "test files" "ARGS A" ["ARGS B" ...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; FILES=$2; shift 2
if [ -n "$FILES" ]; then
  timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
fi
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 600 python bench.py --no-cpu-baseline $a > gpurun_out/${TAG}_b$i.json 2> gpurun_out/${TAG}_b$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "args [$a] rc=$rc"; tail -5 gpurun_out/${TAG}_b$i.err; exit $rc; }
  python3 - "$a" gpurun_out/${TAG}_b$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
print(f"[{sys.argv[1]}]", round(d.get("ms_per_step", 0), 3), {k: round(x["ms"], 3) for k, x in d.get("kernels", {}).items()})
for name, leg in d.get("legs", {}).items():
    print("  leg", name, json.dumps({k: v for k, v in leg.items() if k in ("ms_per_step", "forward_ms", "backward_ms", "contiguous_166", "pitch_168_view", "max_grad_err_over_tolerance")}))
PY
done
