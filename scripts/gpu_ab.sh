#!/bin/bash
# A/B: the default bench (no CPU baseline / legs) once per library variant.
# usage: [BENCH_ARGS="--config c5"] scripts/gpu_ab.sh VARIANT... ("-" = the product libgfd.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  lib=gnn-fraud-detection_amd/gfd/libgfd.so
  [ "$v" != "-" ] && lib=gnn-fraud-detection_amd/gfd/libgfd_$v.so
  GFD_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 10 ${BENCH_ARGS:-} > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err
  rc=$?; echo "ab $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/ab_$v.json')); print('$v', round(d['ms_per_step'],3), {k: round(x['ms'],3) for k,x in d['kernels'].items()})"
done
