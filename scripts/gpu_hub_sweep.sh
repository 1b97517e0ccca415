#!/bin/bash
# Hub threshold / chunk sweep on C4 (tile kernel from GFD_TILE_KERNEL).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for tc in ${TCS:-"16:128" "32:128" "64:128" "128:128"}; do
  t=${tc%%:*}; c=${tc##*:}
  GFD_HUB_THRESHOLD=$t GFD_HUB_CHUNK=$c timeout -k 10 300 python bench.py --steps 6 --warmup 2 --no-cpu-baseline \
      > gpurun_out/hub_${t}_${c}.json 2> gpurun_out/hub_${t}_$c.err || { echo "thr=$t chunk=$c failed"; tail -3 gpurun_out/hub_${t}_$c.err; exit 3; }
  python -c "import json;d=json.load(open('gpurun_out/hub_${t}_${c}.json'));print('thr=$t chunk=$c', round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['layer']['stage_ms'].items()}, 'hubs', d['config']['hubs'])"
done
