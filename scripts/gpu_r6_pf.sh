#!/bin/bash
# Round 6: general slots' next-slot batch-0 prefetch (sl_general NXT).  Parity of the
# tile kernels, then C4 and C5 A / B against the pf0 build (GFD_GENERAL_PF=0).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py tests/test_fullsize_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6p_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6p_tests.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh - pf0 - pf0 || exit 1
BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh - pf0 || exit 1
