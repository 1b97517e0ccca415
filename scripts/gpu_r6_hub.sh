#!/bin/bash
# Round 6: hubs numbered by descending size (chunk launch order).  Hub-touching
# GPU tests, then the headline bench and the 8-way virtual ranks with the hub
# order A / B (GFD_HUB_ORDER=node is the round-5 numbering).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gatconv_gpu.py tests/test_bench_parity_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r6h_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/r6h_tests.txt; [ $rc -eq 0 ] || exit $rc
for o in size node size node; do
  GFD_HUB_ORDER=$o timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 10 > gpurun_out/r6h_ab_$o.json 2> gpurun_out/r6h_ab_$o.err
  rc=$?; [ $rc -eq 0 ] || { echo "bench $o rc=$rc"; tail -5 gpurun_out/r6h_ab_$o.err; exit $rc; }
  python3 -c "import json; d=json.load(open('gpurun_out/r6h_ab_$o.json')); print('$o', round(d['ms_per_step'],3), {k: round(x['ms'],3) for k,x in d['kernels'].items()})"
done
for o in size node; do
  GFD_HUB_ORDER=$o timeout -k 10 400 python scripts/virtual_ranks.py --world 8 --balance cost > gpurun_out/r6h_vr8_$o.json 2> gpurun_out/r6h_vr8_$o.err
  rc=$?; [ $rc -eq 0 ] || { echo "vr $o rc=$rc"; tail -5 gpurun_out/r6h_vr8_$o.err; exit $rc; }
  python3 -c "
import json; d=json.load(open('gpurun_out/r6h_vr8_$o.json'))
print('$o', {k: v for k, v in d.items() if not isinstance(v, (list, dict))})
for r in d.get('ranks', []): print('  ', r)
"
done
