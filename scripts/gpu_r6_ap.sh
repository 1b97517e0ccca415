#!/bin/bash
# Round 6: read-ahead knobs with the bf16 pair rows (gap2: general A fragments 2 k-steps ahead;
# lap3: bf16 light / short light 3 k-steps ahead).  C5 then C4 A / B.
set -u
cd "$(dirname "$0")/.."
BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh - gap2 lap3 - gap2 lap3 || exit 1
bash scripts/gpu_ab.sh - gap2 - gap2 || exit 1
