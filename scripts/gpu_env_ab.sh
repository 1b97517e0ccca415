#!/bin/bash
# Environment A/B of one bench invocation: scripts/gpu_env_ab.sh TAG "BENCH ARGS" "ENV A" "ENV B" ...
# (each ENV a space-separated list of VAR=value, "-" for none); one process per variant.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; ARGS=$2; shift 2
i=0
for e in "$@"; do
  i=$((i+1))
  [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python bench.py --no-cpu-baseline $ARGS > gpurun_out/${TAG}_e$i.json 2> gpurun_out/${TAG}_e$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "env [$e] rc=$rc"; tail -5 gpurun_out/${TAG}_e$i.err; exit $rc; }
  python3 - "$e" gpurun_out/${TAG}_e$i.json <<'PY'
import json, sys
d = json.load(open(sys.argv[2]))
out = {"ms": round(d["ms_per_step"], 3)} if "ms_per_step" in d else {}
for name, leg in d.get("legs", {}).items():
    for k in ("ms_per_step", "forward_ms", "backward_ms"):
        if k in leg:
            out[name + "." + k] = round(leg[k], 3)
print(f"[{sys.argv[1]}]", out)
PY
done
