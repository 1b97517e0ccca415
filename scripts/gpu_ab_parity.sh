#!/bin/bash
# Parity (C4 bench config, sampled, + the 20k-node all-class dropout test) and
# A/B timing of library variants.
# usage: scripts/gpu_ab_parity.sh VARIANT...   ("-" = the product libgfd.so)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
for v in "$@"; do
  lib=gnn-fraud-detection_amd/gfd/libgfd.so
  [ "$v" != "-" ] && lib=gnn-fraud-detection_amd/gfd/libgfd_$v.so
  GFD_LIB_PATH=$PWD/$lib timeout -k 10 400 python -u -m pytest tests/test_bench_parity_gpu.py::test_c4_bench_configuration_sampled_parity tests/test_gatconv_gpu.py::test_dropout_all_classes_at_20k_nodes tests/test_gatconv_gpu.py::test_forward_vs_oracle -x -q --timeout 300 --timeout-method thread > gpurun_out/abp_$v.log 2>&1
  rc=$?; echo "parity $v rc=$rc"; tail -3 gpurun_out/abp_$v.log; [ $rc -eq 0 ] || exit $rc
done
scripts/gpu_ab.sh "$@"
