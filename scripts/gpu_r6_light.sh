#!/bin/bash
# Round 6: the paired-phase light kernel (libgfd_lp1.so: GFD_LIGHT_PAIR=1)
# against the product's k_stream light kernel -- bit-identity of one forward,
# A/B timing, phase profile (libgfd_lpprof.so).  [--tests: the parity suites
# on lp1 first]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=$PWD/gnn-fraud-detection_amd/gfd
timeout -k 10 200 python scripts/dump_fwd.py lp0 || exit $?
GFD_LIB_PATH=$L/libgfd_lp1.so timeout -k 10 200 python scripts/dump_fwd.py pair || exit $?
python scripts/cmp_dumps.py lp0 pair | grep out_
if [ "${1:-}" = "--tests" ]; then
  GFD_LIB_PATH=$L/libgfd_lp1.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py > gpurun_out/r6_tests.txt 2>&1; rc=$?; tail -3 gpurun_out/r6_tests.txt; [ $rc -eq 0 ] || exit $rc
fi
scripts/gpu_ab.sh - lp1 - lp1 || exit $?
GFD_LIB_PATH=$L/libgfd_lpprof.so timeout -k 10 300 python scripts/prof_light_pair.py
