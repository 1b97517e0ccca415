#!/bin/bash
# k_gw change check: backward parity tests, then the C4 fwd + bwd leg under a
# kernel trace (k_gw average) -- product library.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${1:-gw}
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gatconv_gpu.py tests/test_bwd_colmax_gpu.py tests/test_bwd_fused_gpu.py tests/test_models_gpu.py tests/test_dist_gpu.py > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python bench.py --legs-only --legs c4bwd --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/${TAG}_leg.json 2> gpurun_out/${TAG}_leg.err
rc=$?; echo "leg rc=$rc"; exit $rc
