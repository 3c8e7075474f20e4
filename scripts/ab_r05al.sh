#!/bin/bash
# Round-5 A/B: k_primary reads its precomputed candidate masks as wave-uniform values (pmu: scalar loads, a
# wave-uniform candidate walk over scalar-loaded rows instead of a per-lane walk over gathered rows) vs HEAD (-).
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -C oracle > /dev/null || exit 1
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_pmu.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05al_pytest.log 2>&1 || { tail -30 gpurun_out/r05al_pytest.log; exit 1; }
tail -2 gpurun_out/r05al_pytest.log
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c3q c5q c4}" bash scripts/gpu_r04.sh r05al ab - pmu
