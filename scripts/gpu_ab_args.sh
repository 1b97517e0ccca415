#!/bin/bash
# A/B of bench argument sets on the product library: one bench (no CPU
# baseline / legs, 10 steps) per quoted argument string.
# usage: scripts/gpu_ab_args.sh "ARGS A" "ARGS B" ...
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-legs --steps 10 $a > gpurun_out/aba_$i.json 2> gpurun_out/aba_$i.err
  rc=$?; [ $rc -eq 0 ] || { echo "args [$a] rc=$rc"; tail -5 gpurun_out/aba_$i.err; exit $rc; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/aba_$i.json')); print('[$a]', round(d['ms_per_step'],3), {k: round(x['ms'],3) for k,x in d['kernels'].items()})"
done
