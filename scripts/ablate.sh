#!/bin/bash
# tile-kernel ablation: full / aggregation-only / projection-only
cd "$(dirname "$0")/.."
for m in 0 1 2; do
  GFD_FUSED_MODE=$m timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/ablate_$m.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ablate_$m.json'));print('mode $m', d['layer']['stage_ms'])"
done
