#!/bin/bash
# SQ co-execution counters over a short C4 bench (headline line only): how
# often vector and matrix instructions execute together, and the wave states,
# for the tile kernels.  One rocprofv3 pass per group,
# kernel trace only, each under its own limit.
# usage: scripts/gpu_coexec.sh TAG [bench args...]
set -u
cd "$(dirname "$0")/.."
TAG=${1:-coexec}; shift || true
export TMPDIR=/tmp
mkdir -p gpurun_out
P1="SQ_VALU_MFMA_COEXEC_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"
i=0
for c in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-legs "$@" > gpurun_out/${TAG}_p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/${TAG}_p$i.log; exit $rc; }
done
python3 scripts/pmc_coexec.py gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 > gpurun_out/${TAG}_table.txt 2>&1
cat gpurun_out/${TAG}_table.txt
