#!/bin/bash
# Round-5 A/B: the uniform candidate walk (scan_spheres, ILP = false: level 1's reflection scans) with its scalar
# loads one candidate ahead (spf) vs HEAD (-).  Parity first against spf.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -C oracle > /dev/null || exit 1
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_spf.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ak_pytest.log 2>&1 || { tail -30 gpurun_out/r05ak_pytest.log; exit 1; }
tail -2 gpurun_out/r05ak_pytest.log
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c3q c5q c2}" bash scripts/gpu_r04.sh r05ak ab - spf
