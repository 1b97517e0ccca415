#!/bin/bash
# A/B of the hub threshold / chunk (GFD_HUB_THRESHOLD, GFD_HUB_CHUNK) on the C4 bench line.
# usage: scripts/gpu_thr.sh "thr:chunk" ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for tc in "$@"; do
  t=${tc%%:*}; c=${tc##*:}
  GFD_HUB_THRESHOLD=$t GFD_HUB_CHUNK=$c timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 10 > gpurun_out/thr_${t}_${c}.json 2> gpurun_out/thr_${t}_${c}.err
  rc=$?; echo "thr $t chunk $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python3 -c "import json; d=json.load(open('gpurun_out/thr_${t}_${c}.json')); print('$t/$c', round(d['ms_per_step'],3), {k: round(x['ms'],3) for k,x in d['kernels'].items()})"
done
