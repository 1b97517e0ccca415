#!/bin/bash
# bf16 light bound 7 (ABI 9): every GPU test, smoke, then C5 / C4 A/B against
# the bf6 variant (-DGFD_LIGHT_MAX_BF16=6: the round-6 classes).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r6_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r6_smoke.txt; [ $rc -eq 0 ] || exit $rc
BENCH_ARGS="--config c5" scripts/gpu_ab.sh bf6 - bf6 - bf6 - || exit 1
scripts/gpu_ab.sh bf6 - || exit 1
