#!/bin/bash
# Round-5 A/B: the level counts zeroed by k_primary instead of a memset launch (-) vs HEAD before it (base),
# and the dense deep-level arrangement forced for every scene (dense0: RT_DEEP_DENSE_RECORDS=0).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05aa_pytest.log 2>&1 || { tail -30 gpurun_out/r05aa_pytest.log; exit 1; }
tail -1 gpurun_out/r05aa_pytest.log
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_dense0.so timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05aa_pytest_dense0.log 2>&1 || { tail -30 gpurun_out/r05aa_pytest_dense0.log; exit 1; }
tail -1 gpurun_out/r05aa_pytest_dense0.log
REPS=${REPS:-2} BENCH_CFGS="${CFGS:-c3q c3dq c5q}" bash scripts/gpu_r04.sh r05aa ab base - dense0
