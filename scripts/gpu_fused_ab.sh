#!/bin/bash
# Fused backward A/B: the parity tests of k_src_gw (both wave counts), then the
# C4 fwd + bwd leg per GFD_BWD_FUSED value (0 = dh' path, 1 = 8 waves, 2 = 16).
# usage: scripts/gpu_fused_ab.sh TAG [values...]
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=$1; shift
timeout -k 10 600 python -u -m pytest tests/test_bwd_fused_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/${TAG}_tests.txt; [ $rc -eq 0 ] || exit $rc
for v in "$@"; do
  GFD_BWD_FUSED=$v timeout -k 10 300 python bench.py --no-cpu-baseline --legs-only --legs c4bwd > gpurun_out/${TAG}_f$v.json 2> gpurun_out/${TAG}_f$v.err
  rc=$?; [ $rc -eq 0 ] || { echo "fused=$v rc=$rc"; tail -5 gpurun_out/${TAG}_f$v.err; exit $rc; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/${TAG}_f$v.json'))['legs']
for k,l in d.items(): print('fused=$v', k, round(l['forward_ms'],3), round(l['backward_ms'],3))"
done
