#!/bin/bash
# Round-5 closing measurements on one GPU, in parts (each fits one gpurun call):
#   a: every GPU test (one process, per-test limit), smoke()
#   b: rocprofv3 kernel trace + stats of the headline bench; C4 PMC passes
#      (HBM bytes, wave states, instruction mix: scripts/gpu_pmc_all.sh)
#   c: C5 PMC passes (HBM bytes, scripts/gpu_pmc.sh), the default bench line
# usage: GFD_TREE=<git hash> scripts/gpu_final_r5.sh a|b|c
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
case "${1:-a}" in
  a)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_gpu_tests.txt 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r5_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r5_smoke.txt 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r5_smoke.txt; exit $rc ;;
  b)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs > gpurun_out/r5_prof.log 2>&1
    rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
    bash scripts/gpu_pmc_all.sh r5c4 || exit 1
    python3 scripts/pmc_summary.py gpurun_out/r5c4_p1 gpurun_out/r5c4_p2 c4 10000000 50000000 166 1 r5c4 > gpurun_out/r5c4_summary.txt 2>&1
    rc=$?; cat gpurun_out/r5c4_summary.txt; exit $rc ;;
  c)
    CFG="c5 50000000 500000000 166 1" bash scripts/gpu_pmc.sh r5c5 --config c5 || exit 1
    timeout -k 10 900 python bench.py > gpurun_out/r5_bench.json 2> gpurun_out/r5_bench.err
    rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r5_bench.err; exit $rc ;;
esac
