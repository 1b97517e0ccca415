#!/bin/bash
# Round 4: the halo exchange on a 1-GPU box -- gfd_rows_copy parity, bench.Layer's
# sharded path with the halo and all-gather exchanges (emulated collectives),
# and functional rehearsals of the launcher with the halo exchange (gloo, the
# ranks sharing the one GPU; the all-to-all itself runs on the host).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py tests/test_bench_parity_gpu.py::test_bench_multi_rank_path -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_halo_pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -16 gpurun_out/r4_halo_pytest.log; [ $rc -eq 0 ] || exit $rc
for n in 2 4; do
  timeout -k 10 400 python bench.py --gpus $n --rehearse --steps 3 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/r4_rehearse_halo$n.json 2> gpurun_out/r4_rehearse_halo$n.err
  rc=$?; echo "rehearse $n rc=$rc"; tail -3 gpurun_out/r4_rehearse_halo$n.err; [ $rc -eq 0 ] || exit $rc
done
