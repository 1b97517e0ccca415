#!/bin/bash
# Round 4: the N-rank bench path on a 1-GPU box -- parity of bench.Layer's
# sharded path (emulated collectives), a functional 2-rank rehearsal of the
# launcher (gloo, both ranks on the one GPU), and the per-rank compute of 8
# virtual ranks for both shard balances.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_bench_parity_gpu.py::test_bench_multi_rank_path tests/test_gatconv_gpu.py::test_checked_build_accepts_valid_graphs tests/test_gatconv_gpu.py::test_checked_build_rejects_bad_indices -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_dist_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -8 gpurun_out/r4_dist_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 2 --rehearse --steps 3 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/r4_rehearse.json 2> gpurun_out/r4_rehearse.err
rc=$?; echo "rehearse rc=$rc"; tail -3 gpurun_out/r4_rehearse.err; [ $rc -eq 0 ] || exit $rc
for b in nodes messages; do
  timeout -k 10 400 python scripts/virtual_ranks.py --world 8 --balance $b > gpurun_out/r4_vr8_$b.json 2> gpurun_out/r4_vr8_$b.err
  rc=$?; echo "virtual ranks $b rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
