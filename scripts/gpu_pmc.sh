#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 pass per counter group,
# kernel trace only): HBM traffic (FETCH_SIZE, WRITE_SIZE) and SQ wave states.
# usage: scripts/gpu_pmc.sh TAG [bench.py path] [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-pmc}; shift || true
BENCH=${1:-bench.py}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "$SQ"; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python $BENCH --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
