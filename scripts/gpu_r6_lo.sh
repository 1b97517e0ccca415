#!/bin/bash
# Round 6: short light tiles (<= kLightLo messages per slot) in their own k_stream instance
# (fewer rows in flight, deeper A-fragment read-ahead).  Parity, then A / B:
#   lo6ap1 = the round-5 light kernel over the whole class (baseline), loap3 = short tiles
#   with 3 k-steps of A read-ahead, lo4 = the short class up to 4 messages.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py tests/test_fullsize_parity_gpu.py tests/test_dist_gpu.py tests/test_abi.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6l_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6l_tests.txt; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_ab.sh - lo6ap1 loap3 lo4 - lo6ap1 loap3 lo4 || exit 1
BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh - lo6ap1 || exit 1
