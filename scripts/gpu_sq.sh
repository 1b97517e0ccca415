#!/bin/bash
# SQ wave-state counters of the bench kernels (one pass), plus the counter list.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
CTRS=${CTRS:-"SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"}
timeout -k 10 400 rocprofv3 --pmc $CTRS --kernel-trace --output-format csv -d gpurun_out/${TAG:-sq} -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/${TAG:-sq}.log 2>&1
rc=$?; echo "sq rc=$rc"; exit $rc
