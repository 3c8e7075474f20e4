#!/bin/bash
# Round-5 A/B: the BVH levels' persistent grid at 1,024 (g1024: the LDS-resident count, so every workgroup stages the
# BVH once) or 1,536 workgroups (g1536) vs 2,048 (-).  Parity first against g1024.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -C oracle > /dev/null || exit 1
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_g1024.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05an_pytest.log 2>&1 || { tail -30 gpurun_out/r05an_pytest.log; exit 1; }
tail -2 gpurun_out/r05an_pytest.log
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c5q}" bash scripts/gpu_r04.sh r05an ab - g1024 g1536
