#!/bin/bash
# A/B of library variants on bench legs: scripts/gpu_ab_legs2.sh TAG "LEGS" VARIANT... ("-" = product)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; LEGS=$2; shift 2
for v in "$@"; do
  lib=gnn-fraud-detection_amd/gfd/libgfd.so
  [ "$v" != "-" ] && lib=gnn-fraud-detection_amd/gfd/libgfd_$v.so
  GFD_LIB_PATH=$PWD/$lib timeout -k 10 300 python bench.py --no-cpu-baseline --legs-only --legs $LEGS > gpurun_out/${TAG}_$v.json 2> gpurun_out/${TAG}_$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "$v rc=$rc"; tail -5 gpurun_out/${TAG}_$v.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/${TAG}_$v.json'))['legs']
print('$v', {k: (round(l.get('forward_ms', 0), 3), round(l.get('backward_ms', l.get('ms_per_step', 0)), 3)) for k, l in d.items()})"
done
