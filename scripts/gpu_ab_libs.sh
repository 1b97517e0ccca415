#!/bin/bash
# A/B of library builds on C4: bench stage times per libgfd_<variant>.so (VARIANTS env).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=$PWD/gnn-fraud-detection_amd/gfd
for v in ${VARIANTS:-base}; do
  lib=$L/libgfd_$v.so; [ "$v" = base ] && lib=$L/libgfd.so
  GFD_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > gpurun_out/ab_$v.json 2> gpurun_out/ab_$v.err || { echo "$v failed"; tail -5 gpurun_out/ab_$v.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab_$v.json'));print('$v', round(d['ms_per_step'],3), {k: round(x,3) for k,x in d['layer']['stage_ms'].items()})"
done
