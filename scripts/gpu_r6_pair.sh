#!/bin/bash
# Round 6: C5 hub chunks with bf16 rows as 4-B pairs (2 VGPRs a row, 3 batches of 8 in flight;
# nopair = the round-5 path), parity first; then C4 knob A / B (nl4: fp32 general rows a tile
# ahead; wl4: short light W_lo in registers).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_fullsize_parity_gpu.py tests/test_gatconv_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6q_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6q_tests.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh - nopair - nopair || exit 1
bash scripts/gpu_ab.sh - nl4 wl4 - nl4 wl4 || exit 1
