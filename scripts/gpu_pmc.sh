#!/bin/bash
# HBM traffic of the bench's kernels: one rocprofv3 --pmc pass per counter
# (FETCH_SIZE, WRITE_SIZE), kernel trace only, each under its own limit; then
# fold them into profiles/pmc_summary.json (scripts/pmc_summary.py).
# usage: [CFG="c5 50000000 500000000 166 1"] scripts/gpu_pmc.sh TAG [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-pmc}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for c in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; }
done
python3 scripts/pmc_summary.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 ${CFG:-c4 10000000 50000000 166 1} "$TAG" > gpurun_out/${TAG}_summary.txt 2>&1
rc=$?; cat gpurun_out/${TAG}_summary.txt; exit $rc
