#!/bin/bash
# k_bwd_src A/B (round 6, late): bit-identity of the backward against the
# base library, the backward tests, then the C4 fwd+bwd leg per library and a
# kernel-trace of the product's leg.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=$PWD/gnn-fraud-detection_amd/gfd
GFD_LIB_PATH=$L/libgfd_base.so timeout -k 10 300 python scripts/dump_bwd.py bwd_base > gpurun_out/dump_base.txt 2>&1 || { tail -5 gpurun_out/dump_base.txt; exit 1; }
timeout -k 10 300 python scripts/dump_bwd.py bwd_new > gpurun_out/dump_new.txt 2>&1 || { tail -5 gpurun_out/dump_new.txt; exit 1; }
python scripts/cmp_dumps.py bwd_base bwd_new
timeout -k 10 900 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bwd_colmax_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/src_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/src_tests.txt; [ $rc -eq 0 ] || exit $rc
LEGS=c4bwd scripts/gpu_ab_legs.sh base - base - || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_src -o run -- python bench.py --no-cpu-baseline --steps 5 --warmup 2 --legs c4bwd > gpurun_out/prof_src.log 2>&1 || { tail -5 gpurun_out/prof_src.log; exit 1; }
echo done
