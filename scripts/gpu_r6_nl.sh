#!/bin/bash
# Round 6: general fp32 slots with rows a tile ahead (nl4 / nl2: GFD_GENERAL_NL_F32 -- spill-free
# since the two slots share their batch registers) and the short light instance with W_lo of 4
# more k-steps in registers (wl4: GFD_LIGHT_LO_WL=4).  C4 A / B, then C5 for wl4.
set -u
cd "$(dirname "$0")/.."
bash scripts/gpu_ab.sh - nl4 wl4 nl2 - nl4 wl4 nl2 || exit 1
BENCH_ARGS="--config c5" bash scripts/gpu_ab.sh - wl4 || exit 1
