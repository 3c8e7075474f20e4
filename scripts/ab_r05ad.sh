#!/bin/bash
# Round-5 A/B: the sphere test's nearer root alone (root: T1 = (-B - sq)/2 is lists:min([T0, T1]) and both roots
# are >= 0 iff T1 is) and, on top, the occluder walk's list position read on exact ties only with the row taken
# from the chunk's uniform base (rt) vs HEAD (-).  First the parity tests against the rt variant.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -C oracle > /dev/null || exit 1
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_rt.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ad_pytest.log 2>&1 || { tail -30 gpurun_out/r05ad_pytest.log; exit 1; }
tail -2 gpurun_out/r05ad_pytest.log
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c3q c5q}" bash scripts/gpu_r04.sh r05ad ab - root rt
