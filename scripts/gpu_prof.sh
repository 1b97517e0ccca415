#!/bin/bash
# rocprofv3 kernel-trace summary of the default bench (CSV under gpurun_out/$1)
set -u
cd "$(dirname "$0")/.."
OUT=gpurun_out/${1:-prof}
shift || true
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
