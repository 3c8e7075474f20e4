#!/bin/bash
# Round-5 A/B: inline chain walks (k_reflect_shade walks the chains of the records it finds terminal, and
# the deepest level's launch shades its hits instead of queueing them) vs the build before (base).
#   bash scripts/ab_r05z.sh test   GPU parity (frames, full-size, parity, knobs) + the RT_DEBUG_LISTS run
#   bash scripts/ab_r05z.sh ab     configs 3 and 5, base vs the default build
set -o pipefail
mkdir -p gpurun_out
if [ "$1" = test ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05z_pytest.log 2>&1 || { tail -30 gpurun_out/r05z_pytest.log; exit 1; }
  tail -2 gpurun_out/r05z_pytest.log
  bash scripts/debug_lists.sh run > gpurun_out/r05z_debug_lists.log 2>&1 || { tail -30 gpurun_out/r05z_debug_lists.log; exit 1; }
  tail -2 gpurun_out/r05z_debug_lists.log
else
  REPS=${REPS:-2} BENCH_CFGS="${CFGS:-c3q c3dq c5q}" bash scripts/gpu_r04.sh r05z ab base -
fi
