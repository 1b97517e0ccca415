#!/bin/bash
# tile kernel occupancy A/B (GFD_FUSED_OCC 8 vs 4) at F = 166, 128, 64
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 2
for F in ${FS:-166 128 64}; do
  for o in ${OCCS:-8 4}; do
    GFD_FUSED_OCC=$o timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --features $F > gpurun_out/occ_${F}_$o.json 2> gpurun_out/occ_${F}_$o.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/occ_${F}_$o.json'));print('F=$F occ=$o', round(d['ms_per_step'],2), {k:round(v,2) for k,v in d['layer']['stage_ms'].items()})"
  done
done
