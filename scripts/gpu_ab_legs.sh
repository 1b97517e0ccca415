#!/bin/bash
# A/B of bench legs (no headline CPU baseline) per library variant.
# usage: LEGS=c4bwd,c2 scripts/gpu_ab_legs.sh VARIANT... ("-" = the product libgfd.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  lib=gnn-fraud-detection_amd/gfd/libgfd.so
  [ "$v" != "-" ] && lib=gnn-fraud-detection_amd/gfd/libgfd_$v.so
  GFD_LIB_PATH=$PWD/$lib timeout -k 10 400 python bench.py --no-cpu-baseline --steps 5 --warmup 2 --legs ${LEGS:-c4bwd} > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err
  rc=$?; echo "abl $v rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/abl_$v.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/abl_$v.json')); print('$v', {k: (round(x['ms_per_step'],3) if x.get('ms_per_step') else None, round(x.get('backward_ms',0),3)) for k,x in d['legs'].items()})"
done
