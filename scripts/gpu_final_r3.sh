#!/bin/bash
# Round-3 closing measurements on one GPU, in two parts (each fits one gpurun call):
#   part a: the backward NaN-padding parity test, C4 forward PMC passes
#           (scripts/gpu_pmc_all.sh), a rocprofv3 kernel-trace of the headline bench
#   part b: C5 forward PMC passes (scripts/gpu_pmc.sh), the default bench line
# usage: scripts/gpu_final_r3.sh a|b
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ "${1:-a}" = a ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bench_parity_gpu.py -k backward_nan > gpurun_out/r3c_nanbwd.txt 2>&1
  rc=$?; echo "nan-test rc=$rc"; tail -2 gpurun_out/r3c_nanbwd.txt; [ $rc -eq 0 ] || exit $rc
  bash scripts/gpu_pmc_all.sh r3c || exit 1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3c_prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs > gpurun_out/r3c_prof.log 2>&1
  rc=$?; echo "prof rc=$rc"; exit $rc
else
  CFG="c5 50000000 500000000 166 1" bash scripts/gpu_pmc.sh r3c5 --config c5 || exit 1
  timeout -k 10 900 python bench.py > gpurun_out/r3c_bench.json 2> gpurun_out/r3c_bench.err
  rc=$?; echo "bench rc=$rc"; exit $rc
fi
