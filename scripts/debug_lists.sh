#!/bin/bash
# The chain-link diagnostic build (-DRT_DEBUG_LISTS: k_walk / k_walk_deep print and trap on a
# parent link outside its level, a colour entry whose link word is not its record's, or a parent
# record of another pixel) and the wavefront-path tests run against it.
#   build (here, no GPU):  bash scripts/debug_lists.sh build
#   run (on the GPU box):  bash scripts/debug_lists.sh run
set -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
LIB=$ROOT/eraytracer_amd/variants/librtmi355x_debug_lists.so
if [ "${1:-build}" = build ]; then
  make -s -C "$ROOT/eraytracer_amd/csrc" variant NAME=debug_lists DEFS="-DRT_DEBUG_LISTS" && ls -l "$LIB"
else
  test -f "$LIB" || { echo "missing $LIB: build it first"; exit 1; }
  mkdir -p "$ROOT/gpurun_out"
  cd "$ROOT" && RT_LIB_PATH=$LIB timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
    "tests/test_gpu_fullsize.py::test_fused_wavefront_kernels_all_paths" \
    "tests/test_gpu_frames.py::test_fused_path_across_regrowth_and_partial_groups" \
    "tests/test_gpu_frames.py::test_fused_path_with_row_passes" \
    "tests/test_gpu_fullsize.py::test_bvh_forced_on_every_level_and_scene" \
    "tests/test_gpu_fullsize.py::test_config5_rows_through_the_bvh_path" \
    "tests/test_gpu_fullsize.py::test_inline_walks_dense_deep_levels" \
    "tests/test_gpu_limits.py"
fi
