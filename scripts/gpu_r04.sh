#!/bin/bash
# Round-4 GPU steps on one MI355X (each step under its own time limit, stopped at the first failure):
#   bash scripts/gpu_r04.sh TAG tests "pytest -k expr"   selected GPU tests
#   bash scripts/gpu_r04.sh TAG suite                    the whole GPU suite
#   bash scripts/gpu_r04.sh TAG bench [c2 c3 c3d c4 c5]  bench lines (c3d: the driver's 20/5 steps)
#   bash scripts/gpu_r04.sh TAG ab VARIANT...            A/B of library variants (eraytracer_amd/variants/
#                                                        librtmi355x_NAME.so via RT_LIB_PATH; "-" = the default build;
#                                                        "env:VAR=value" = the default build with that environment)
#                                                        on configs BENCH_CFGS (default "c3 c5")
set -o pipefail
TAG=${1:-r04}; MODE=${2:-bench}; shift 2 || true
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--scene default --width 1920 --height 1080 --depth 5"
C5="--scene s256 --depth 8 --spp 16"
cfg_args() {
  case $1 in
    c2) echo "$C2 --no-cpu-baseline --no-boundary" ;;
    c3) echo "" ;;
    c3d) echo "--steps 20 --warmup 5" ;;
    c3q) echo "--no-cpu-baseline --no-boundary" ;;
    c3q3) echo "--no-cpu-baseline --no-boundary --inflight 3" ;;
    c3q6) echo "--no-cpu-baseline --no-boundary --inflight 6" ;;
    c3dq) echo "--steps 20 --warmup 5 --no-cpu-baseline --no-boundary" ;;
    c4) echo "--size 8192 --no-cpu-baseline --no-boundary" ;;
    c5) echo "$C5 --steps 10 --warmup 4 --no-boundary --cpu-seconds 10" ;;
    c5q) echo "$C5 --steps 8 --warmup 3 --no-boundary --no-cpu-baseline" ;;
  esac
}
line() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline',{})
print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame', 'dom', r.get('launch_ms_live'), 'frac', r.get('frac'))" "$1" "$2"; }
case $MODE in
  tests)
    make -C oracle > /dev/null || exit 1
    timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread -k "$1" \
      > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
    grep -E "PASSED|FAILED|ERROR|passed|failed|max \|delta\||filtered" gpurun_out/pytest_$TAG.log | tail -40; exit $rc ;;
  suite)
    make -C oracle > /dev/null || exit 1
    timeout -k 10 1000 python -u -m pytest tests -x -v -m gpu --timeout 600 --timeout-method thread \
      > gpurun_out/pytest_$TAG.log 2>&1; rc=$?
    tail -3 gpurun_out/pytest_$TAG.log; exit $rc ;;
  bench)
    make -C oracle > /dev/null || exit 1
    for c in "$@"; do
      timeout -k 10 300 python bench.py $(cfg_args $c) > gpurun_out/${TAG}_bench_$c.json 2> gpurun_out/${TAG}_bench_$c.err \
        || { tail -5 gpurun_out/${TAG}_bench_$c.err; exit 1; }
      line gpurun_out/${TAG}_bench_$c.json $c || exit 1
    done ;;
  ab)
    : > gpurun_out/${TAG}_ab.txt
    for rep in $(seq 1 ${REPS:-2}); do
      for c in ${BENCH_CFGS:-c3q c5q}; do
        for v in "$@"; do
          lib=""; ev=""
          case $v in -) ;; env:*) ev=$(echo ${v#env:} | tr , " ") ;; *) lib="eraytracer_amd/variants/librtmi355x_$v.so" ;; esac
          env $ev RT_LIB_PATH=$lib timeout -k 10 300 python bench.py $(cfg_args $c) > gpurun_out/${TAG}_ab_one.json 2> gpurun_out/${TAG}_ab_one.err \
            || { tail -5 gpurun_out/${TAG}_ab_one.err; exit 1; }
          line gpurun_out/${TAG}_ab_one.json "$c $v rep$rep" | tee -a gpurun_out/${TAG}_ab.txt || exit 1
        done
      done
    done ;;
esac
