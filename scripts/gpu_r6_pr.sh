#!/bin/bash
# Round 6: bf16 tile-kernel rows held as RowL pairs (2 VGPRs a row).  Parity (fp32 paths too:
# the FMA helpers were rewritten), then C5 A / B: nopr = 3-VGPR rows (before), p8 = pairs with
# the whole batch 0 of a general slot (8 rows) issued a tile ahead.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 800 python -u -m pytest tests/test_fullsize_parity_gpu.py tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6r_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6r_tests.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh - nopr p8 - nopr p8 || exit 1
# phase split of the tile loops (diagnostic -DGFD_PROF build, per-wave s_memtime stamps)
GFD_LIB_PATH=$PWD/gnn-fraud-detection_amd/gfd/libgfd_prof.so timeout -k 10 300 python scripts/prof_phases.py > gpurun_out/r6r_phases.txt 2>&1
rc=$?; echo "phases rc=$rc"; cat gpurun_out/r6r_phases.txt | tail -20; exit $rc
