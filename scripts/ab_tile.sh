#!/bin/bash
# A/B the tile kernels: parity tests under the persistent kernel, then bench both
# at F = 166 / 128 / 64 (feature-chunk classes 3 / 2 / 1).
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 120 python -c "import __graft_entry__ as g; g.build()" > gpurun_out/build.log 2>&1 || exit 2
GFD_TILE_KERNEL=${TK:-2} timeout -k 10 600 python -m pytest tests/test_gatconv_gpu.py -m gpu -q -x > gpurun_out/pytest_persist.log 2>&1
rc=$?; echo "pytest(persist) rc=$rc"; tail -15 gpurun_out/pytest_persist.log
[ $rc -le 1 ] || exit $rc
for F in 166 128 64; do
  for k in 1 ${TK:-2}; do
    GFD_TILE_KERNEL=$k timeout -k 10 300 python bench.py --steps 8 --warmup 2 --no-cpu-baseline --features $F > gpurun_out/ab_${F}_$k.json 2> gpurun_out/ab_${F}_$k.err || exit $?
    python -c "import json;d=json.load(open('gpurun_out/ab_${F}_$k.json'));print('F=$F kernel=$k', d['ms_per_step'], d['layer']['stage_ms'])"
  done
done
