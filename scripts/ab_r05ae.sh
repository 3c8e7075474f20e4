#!/bin/bash
# Round-5 A/B: rt (nearer root + ties-only list positions, r05ad) vs rt2 (the tie branch on the bare t == t*
# ballot) vs tie (ties-only list positions without the root change) vs HEAD (-).  Parity first against rt2.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -C oracle > /dev/null || exit 1
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_rt2.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ae_pytest.log 2>&1 || { tail -30 gpurun_out/r05ae_pytest.log; exit 1; }
tail -2 gpurun_out/r05ae_pytest.log
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c3q c5q}" bash scripts/gpu_r04.sh r05ae ab - rt rt2 tie
