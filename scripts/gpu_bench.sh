#!/bin/bash
# Short bench + rocprofv3 kernel-trace summary of the same command.
# usage: scripts/gpu_bench.sh TAG [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-dev}; shift || true
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err
rc=$?; echo "bench rc=$rc"; tail -5 gpurun_out/bench_$TAG.err; cat gpurun_out/bench_$TAG.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python bench.py "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
