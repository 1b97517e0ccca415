#!/bin/bash
# PMC passes over a short C4 bench (headline line only): HBM traffic
# (FETCH_SIZE, WRITE_SIZE) and two SQ groups (wave states; instruction mix).
# One rocprofv3 pass per group, kernel trace only, each under its own limit.
# usage: scripts/gpu_pmc_all.sh TAG [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-pmc}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for c in "FETCH_SIZE" "WRITE_SIZE" "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; }
done
python3 scripts/pmc_table.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 gpurun_out/${TAG}_p3 gpurun_out/${TAG}_p4 > gpurun_out/${TAG}_table.txt 2>&1
cat gpurun_out/${TAG}_table.txt
