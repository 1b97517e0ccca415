#!/bin/bash
# Counters of the C4 forward + backward leg (bench.py --legs c4bwd): HBM bytes
# (FETCH_SIZE, WRITE_SIZE) and two SQ passes (wave states; instruction mix),
# one rocprofv3 --pmc pass each, kernel trace only, each under its own limit.
# Output: gpurun_out/${TAG}_{fetch,write,sq1,sq2}/run_counter_collection.csv
set -u
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${TAG:-bwdpmc}
P_fetch="FETCH_SIZE"
P_write="WRITE_SIZE"
P_sq1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU"
P_sq2="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES"
for p in fetch write sq1 sq2; do
  v=P_$p
  timeout -s KILL 200 rocprofv3 --pmc ${!v} --kernel-trace --output-format csv -d gpurun_out/${T}_$p -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --legs-only --legs c4bwd > gpurun_out/${T}_$p.log 2>&1
  rc=$?; echo "pass $p rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${T}_$p.log; exit $rc; }
done
