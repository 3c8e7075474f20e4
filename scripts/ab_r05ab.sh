#!/bin/bash
# Round-5 A/B: inline walks with every level shaded by its own launch (dense arrangement) — no k_walk, no deepest
# k_items (-) vs HEAD before it (base).  First the GPU suite and the RT_DEBUG_LISTS run.
set -o pipefail
mkdir -p gpurun_out
bash scripts/gpu_r05.sh r05ab test || exit 1
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c3q c3dq c5q}" bash scripts/gpu_r04.sh r05ab ab base -
