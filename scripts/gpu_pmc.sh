#!/bin/bash
# HBM traffic of the bench kernels: one rocprofv3 pass per TCC counter group
# (FETCH_SIZE and WRITE_SIZE do not fit one pass), kernel trace only.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 400 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/pmc_$c -o run -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/pmc_$c.log 2>&1
  rc=$?; echo "pmc $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
