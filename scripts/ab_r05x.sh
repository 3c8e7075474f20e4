#!/bin/bash
# Round-5 A/B: the chain walk re-forming parents' light terms from kept (dd, sp) pairs (terms) vs HEAD (base)
set -o pipefail
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_terms.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05x_pytest.log 2>&1 || { tail -30 gpurun_out/r05x_pytest.log; exit 1; }
tail -2 gpurun_out/r05x_pytest.log
bash scripts/debug_lists.sh run > gpurun_out/r05x_debug_lists.log 2>&1 || { tail -30 gpurun_out/r05x_debug_lists.log; exit 1; }
tail -1 gpurun_out/r05x_debug_lists.log
REPS=3 BENCH_CFGS="c3q c3dq c5q" bash scripts/gpu_r04.sh r05x ab base terms
