#!/bin/bash
# tile-kernel ablation: full / aggregation-only / projection-only, per feature width
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 2
for F in ${FS:-166 64}; do
  for m in 0 1 2; do
    GFD_FUSED_MODE=$m timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --features $F "$@" > gpurun_out/ablate_${F}_$m.json 2>/dev/null || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ablate_${F}_$m.json'));print('F=$F mode $m', {k:round(v,2) for k,v in d['layer']['stage_ms'].items()})"
  done
done
