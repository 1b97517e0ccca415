#!/bin/bash
# Multi-rank rehearsal on the 1-GPU box (gloo host-staged exchange, ranks
# sharing the card): bench.py's own launcher at N = 2, and the driver's
# torch.distributed.run form at N = 4.  Not a scaling measurement.
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --gpus 2 --rehearse --steps 3 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/r6_rehearse2.json 2> gpurun_out/r6_rehearse2.err
rc=$?; echo "rehearse 2 rc=$rc"; tail -2 gpurun_out/r6_rehearse2.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --rehearse --steps 3 --warmup 1 --no-legs --no-cpu-baseline > gpurun_out/r6_rehearse4.json 2> gpurun_out/r6_rehearse4.err
rc=$?; echo "rehearse 4 rc=$rc"; tail -2 gpurun_out/r6_rehearse4.err; exit $rc
