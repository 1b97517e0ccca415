#!/bin/bash
# Two SQ counter passes (wave states; instruction mix) for the current tile kernel
# selection (GFD_TILE_KERNEL from the environment); output under gpurun_out/$TAG_*.
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-sq}
[ -f gpurun_out/counters.txt ] || timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1 || true
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
P2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $P --kernel-trace --output-format csv -d gpurun_out/${T}_$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/${T}_$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_$i.log; exit $rc; }
done
