#!/bin/bash
# GPU parity tests (one process, per-test time limit), then a short bench.
# usage: scripts/gpu_tests.sh [pytest -k expression]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
K=${1:-}
ARGS=(-u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider)
[ -n "$K" ] && ARGS+=(-k "$K")
timeout -k 10 900 python "${ARGS[@]}" > gpurun_out/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -30 gpurun_out/pytest.log; exit $rc
