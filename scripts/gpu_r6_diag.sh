#!/bin/bash
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=$PWD/gnn-fraud-detection_amd/gfd
GFD_LIB_PATH=$L/libgfd_lp0.so timeout -k 10 200 python scripts/dump_fwd.py lp0 || exit $?
GFD_LIB_PATH=$L/libgfd_lpw.so timeout -k 10 200 python scripts/dump_fwd.py lpw || exit $?
GFD_LIB_PATH=$L/libgfd_lpp.so timeout -k 10 200 python scripts/dump_fwd.py lpp || exit $?
timeout -k 10 200 python scripts/dump_fwd.py pair || exit $?
timeout -k 10 200 python scripts/dump_fwd.py pair2 || exit $?
for v in lpw lpp pair pair2; do echo "== lp0 vs $v"; python scripts/cmp_dumps.py lp0 $v | grep out_; done
