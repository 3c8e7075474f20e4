#!/bin/bash
# Round-5 A/B: inline chain walks, register-allocation variants (iwA: walk inputs re-read from the
# kernel-argument segment; iwB: + iw tested where used; iwC: + the record's tail re-read) vs the first
# inline-walk build (the default library here) and the build before inline walks (base)
set -o pipefail
mkdir -p gpurun_out
for v in iwA iwC; do
  RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05z2_pytest_$v.log 2>&1 || { tail -30 gpurun_out/r05z2_pytest_$v.log; exit 1; }
  tail -1 gpurun_out/r05z2_pytest_$v.log
done
REPS=${REPS:-2} BENCH_CFGS="${CFGS:-c3q c3dq c5q}" bash scripts/gpu_r04.sh r05z2 ab base - iwA iwB iwC
