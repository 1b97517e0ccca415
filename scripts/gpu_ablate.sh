#!/bin/bash
# Tile-stage ablation on C4: full / aggregation-only / projection-only (GFD_FUSED_MODE),
# optionally over occupancy settings.  Outputs are wrong in modes 1 and 2.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for occ in ${OCCS:-4}; do
for m in ${MODES:-0 1 2}; do
  tag=m${m}_o${occ}_tk${TK:-0}
  GFD_TILE_KERNEL=${TK:-0} GFD_FUSED_OCC=$occ GFD_FUSED_MODE=$m timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline ${BENCH_EXTRA:-} \
      > gpurun_out/abl_$tag.json 2> gpurun_out/abl_$tag.err || { echo "$tag failed"; tail -5 gpurun_out/abl_$tag.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/abl_$tag.json'));print('$tag', round(d['ms_per_step'],3), d['layer']['stage_ms'])"
done; done
