#!/bin/bash
# Round-6 closing measurements on one GPU, in parts (each fits one gpurun call):
#   a: every GPU test (one process, per-test limit), smoke()
#   b: rocprofv3 kernel trace + stats of the headline bench; C4 PMC passes
#      (HBM bytes, wave states, instruction mix: scripts/gpu_pmc_all.sh)
#   c: C5 PMC passes (HBM bytes), the default bench line (legs + CPU baseline)
#   d: 8-way virtual ranks (forward), backward PMC passes
# The PMC CSVs come back under gpurun_out/; fold them into profiles/pmc_summary.json
# here with scripts/pmc_summary.py (GFD_TREE=<git hash>).
#   e: the default bench line alone
# usage: scripts/gpu_final_r6.sh a|b|c|d|e
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
case "${1:-a}" in
  a)
    timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > gpurun_out/r6_gpu_tests.txt 2>&1
    rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/r6_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6_smoke.txt 2>&1
    rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/r6_smoke.txt; exit $rc ;;
  b)
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r6_prof -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-legs > gpurun_out/r6_prof.log 2>&1
    rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
    bash scripts/gpu_pmc_all.sh r6c4; exit $? ;;
  c)
    # the fold on the box rewrites its copy of profiles/pmc_summary.json, which
    # the bench line reads for roofline.traffic: keep the committed one
    cp profiles/pmc_summary.json /tmp/pmc_keep.json
    CFG="c5 50000000 500000000 166 1" bash scripts/gpu_pmc.sh r6c5 --config c5 || exit 1
    cp /tmp/pmc_keep.json profiles/pmc_summary.json
    timeout -k 10 900 python bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err
    rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r6_bench.err; exit $rc ;;
  e)
    timeout -k 10 900 python bench.py > gpurun_out/r6_bench.json 2> gpurun_out/r6_bench.err
    rc=$?; echo "bench rc=$rc"; tail -3 gpurun_out/r6_bench.err; exit $rc ;;
  d)
    timeout -k 10 400 python scripts/virtual_ranks.py --world 8 --balance cost > gpurun_out/r6_vr8.json 2> gpurun_out/r6_vr8.err
    rc=$?; echo "vr8 rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/r6_vr8.err; exit $rc; }
    TAG=r6bwd bash scripts/gpu_bwd_pmc.sh; exit $? ;;
esac
