#!/bin/bash
# k_bwd_msg phase ablation: kernel-trace stats of the C4 fwd+bwd leg per library variant.
# usage: scripts/gpu_bwd_ablate.sh VARIANT... ("-" = the product libgfd.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  lib=gnn-fraud-detection_amd/gfd/libgfd.so
  [ "$v" != "-" ] && lib=gnn-fraud-detection_amd/gfd/libgfd_$v.so
  export GFD_LIB_PATH=$PWD/$lib
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abl_$v -o run -- python bench.py --legs-only --legs c4bwd --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/abl_$v.json 2> gpurun_out/abl_$v.err
  rc=$?; echo "ablate $v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
