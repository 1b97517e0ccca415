#!/bin/bash
# Quick GPU check: selected test files (one process, per-test limit), then the
# headline bench (no CPU baseline / legs).
# usage: scripts/gpu_quick.sh TAG "tests/a.py tests/b.py" [-k expr]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; FILES=$2; shift 2
timeout -k 10 900 python -u -m pytest $FILES -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider "$@" > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 10 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_bench.err; exit $rc; }
python3 -c "import json; d=json.load(open('gpurun_out/${TAG}_bench.json')); print(round(d['ms_per_step'],3), {k: round(x['ms'],3) for k,x in d['kernels'].items()})"
