#!/bin/bash
# One iteration on the GPU box: checked-build scenarios, GPU tests, phase profile,
# bench.  Stops at the first failure.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
L=$PWD/gnn-fraud-detection_amd/gfd
GFD_LIB_PATH=$L/libgfd_chk.so timeout -k 10 200 python scripts/chk_run.py > gpurun_out/chk.log 2>&1
rc=$?; grep -c "site=0 value=0" gpurun_out/chk.log; grep "max err" gpurun_out/chk.log | tr "\n" " "; echo; grep "site=[1-9]" gpurun_out/chk.log | head -5; [ $rc -eq 0 ] || { tail -20 gpurun_out/chk.log; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A30 "Error\|FAIL" gpurun_out/pytest_gpu.log | head -60; exit $rc; }
GFD_LIB_PATH=$L/libgfd_prof.so GFD_PROF_DUMP=1 timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof.json 2> gpurun_out/prof.err
rc=$?; grep "\[bench\] k_stream" gpurun_out/prof.err; [ $rc -eq 0 ] || { tail -5 gpurun_out/prof.err; exit $rc; }
timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/b.json 2> gpurun_out/b.err
rc=$?; [ $rc -eq 0 ] || { tail -5 gpurun_out/b.err; exit $rc; }
python -c "import json;d=json.load(open('gpurun_out/b.json'));print(round(d['ms_per_step'],3), {k: round(v,3) for k,v in d['layer']['stage_ms'].items()}, round(d['roofline']['frac'],4))"
