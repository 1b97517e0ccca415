#!/bin/bash
# A/B every tile kernel variant on C4 (F = 166): one bench per GFD_TILE_KERNEL value.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for k in ${TKS:-0 2 3 4}; do
  GFD_TILE_KERNEL=$k timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_EXTRA:-} \
      > gpurun_out/ab_tk$k.json 2> gpurun_out/ab_tk$k.err || { echo "tk=$k failed rc=$?"; tail -5 gpurun_out/ab_tk$k.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/ab_tk$k.json'));print('tk=$k', round(d['ms_per_step'],3), d['layer']['stage_ms'])"
done
