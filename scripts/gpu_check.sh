#!/bin/bash
# One GPU session: tests, smoke, bench.  Stops at the first crash/timeout
# (exit >= 124 or signal), continues past ordinary test failures (exit 1).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -30 gpurun_out/build.log; exit 2; }
timeout -k 10 ${PYTEST_TIMEOUT:-900} python -m pytest tests -m "${PYTEST_MARK:-gpu}" -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -40 gpurun_out/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.build(); g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -5 gpurun_out/smoke.log
ok $rc || exit $rc
if [ -n "${BENCH_ARGS+x}" ]; then
  timeout -k 10 600 python bench.py $BENCH_ARGS > gpurun_out/bench.json 2> gpurun_out/bench.err
  rc=$?; echo "bench rc=$rc"; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err
fi
