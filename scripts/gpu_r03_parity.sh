#!/bin/bash
# Round 3: whole-frame parity (oracle) and filters == brute force, then a short bench line.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1000 python -u -m pytest tests/test_gpu_frames.py \
    "tests/test_gpu_fullsize.py::test_general_pow_and_mixed_scenes" -v -s --timeout 700 --timeout-method thread \
    2>&1 | tee gpurun_out/r03_parity.log
