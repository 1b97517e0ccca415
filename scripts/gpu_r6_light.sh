#!/bin/bash
# Round 6: the paired-phase light kernel -- probe, bit-identity against the
# k_stream light kernel (libgfd_lp0.so), parity tests, A/B timing.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out

GFD_LIB_PATH=$PWD/gnn-fraud-detection_amd/gfd/libgfd_lp0.so timeout -k 10 200 python scripts/dump_fwd.py lp0 || exit $?
timeout -k 10 200 python scripts/dump_fwd.py pair || exit $?
python scripts/cmp_dumps.py lp0 pair
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py > gpurun_out/r6_tests.txt 2>&1; rc=$?; tail -5 gpurun_out/r6_tests.txt; [ $rc -eq 0 ] || exit $rc
scripts/gpu_ab.sh lp0 - lp0 -
