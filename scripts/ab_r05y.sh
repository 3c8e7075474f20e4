#!/bin/bash
# Round-5 A/B: shadow tests without the target's own distance when no lane has an occluder candidate (tstar) vs HEAD
set -o pipefail
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_tstar.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05y_pytest.log 2>&1 || { tail -30 gpurun_out/r05y_pytest.log; exit 1; }
tail -2 gpurun_out/r05y_pytest.log
REPS=3 BENCH_CFGS="c3q c3dq" bash scripts/gpu_r04.sh r05y ab base tstar
