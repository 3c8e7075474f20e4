#!/bin/bash
# Round-5 A/B: the occluder walk software-pipelined (opf: the next candidate's row loaded while the current one is
# tested) vs HEAD (-).  Parity first against opf.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
make -C oracle > /dev/null || exit 1
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_opf.so timeout -k 10 900 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_knobs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05ai_pytest.log 2>&1 || { tail -30 gpurun_out/r05ai_pytest.log; exit 1; }
tail -2 gpurun_out/r05ai_pytest.log
REPS=${REPS:-3} BENCH_CFGS="${CFGS:-c5q c3q}" bash scripts/gpu_r04.sh r05ai ab - opf
