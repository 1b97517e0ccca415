#!/bin/bash
# Round evidence on one GPU: tests, smoke, rocprofv3 kernel stats, PMC traffic
# passes and the default bench (with the CPU baseline).  Stops at the first
# crash / timeout.
set -u
cd "$(dirname "$0")/.."
TAG=${1:-r1}
PYTEST_MARK=gpu bash scripts/gpu_check.sh || exit $?
bash scripts/gpu_prof.sh prof_$TAG || exit $?
bash scripts/gpu_pmc.sh || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench_$TAG.json; exit $rc
