#!/bin/bash
# Logits-pass A/B (round 6, late): parity of the product, then the headline
# bench per library (C4 twice, then C5 twice).  usage: scripts/gpu_r6_lg.sh VARIANT...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/lg_tests.txt 2>&1
rc=$?; echo "pytest product rc=$rc"; tail -3 gpurun_out/lg_tests.txt; [ $rc -eq 0 ] || exit $rc
scripts/gpu_ab.sh "$@" "$@" || exit 1
BENCH_ARGS="--config c5" scripts/gpu_ab.sh "$@" "$@" || exit 1
