#!/bin/bash
# Round 4: the phased halo exchange -- every GPU test, smoke, launcher
# rehearsals (gloo, ranks sharing the one GPU), 8 virtual ranks (cost balance).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r4_gpu_tests.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_smoke.txt 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/r4_smoke.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 4 --rehearse --steps 3 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/r4_rehearse_halo4.json 2> gpurun_out/r4_rehearse_halo4.err
rc=$?; echo "rehearse rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python scripts/virtual_ranks.py --world 8 --balance cost > gpurun_out/r4_vr8_final.json 2> gpurun_out/r4_vr8_final.err
rc=$?; echo "virtual ranks rc=$rc"; exit $rc
