#!/bin/bash
# Round-6 GPU steps (each under its own time limit; the first failure ends the call).
#   bash scripts/gpu_r06.sh TAG lim       the input-size tests (depth, lights, objects) alone
#   VARIANTS="- a b" CFGS="c3dq c5q" REPS=2 bash scripts/gpu_r06.sh TAG ab   A/B of library variants
#   bash scripts/gpu_r06.sh TAG test      GPU parity suite, then the RT_DEBUG_LISTS build's wavefront tests
#   bash scripts/gpu_r06.sh TAG bench     bench lines: config 3 (driver-style 20/5 and default), configs 2, 5
#   bash scripts/gpu_r06.sh TAG c3        config 3 driver-style bench line only
#   bash scripts/gpu_r06.sh TAG setup     config 3 lines with the setup leg (8 and 4 HW queues), config 5's, the N = 8 floor
#   bash scripts/gpu_r06.sh TAG prof3     rocprofv3 kernel trace + PMC passes of config 3
#   bash scripts/gpu_r06.sh TAG prof5     the same for config 5 (prof2: config 2)
#   VARIANTS="- a b" [PMCV_ARGS=...] bash scripts/gpu_r06.sh TAG pmcv   instruction counts per kernel of variants
set -o pipefail
TAG=${1:-r06}
PART=${2:-test}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--scene default --width 1920 --height 1080 --depth 5"
C5="--scene s256 --depth 8 --spp 16"
b() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench_$name.json 2> gpurun_out/${TAG}_bench_$name.err || { tail -5 gpurun_out/${TAG}_bench_$name.err; exit 1; }; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame', 'dom', r.get('launch_ms_live'), 'frac', r.get('frac'), 'cpu', d.get('cpu_baseline', {}).get('value'), d.get('cpu_baseline', {}).get('cores'))" gpurun_out/${TAG}_bench_$name.json $name; }
cfg_args() {
  case $1 in
    c2q) echo "$C2 --no-cpu-baseline --no-boundary --no-setup" ;;
    c3q) echo "--no-cpu-baseline --no-boundary --no-setup" ;;
    c3dq) echo "--steps 20 --warmup 5 --no-cpu-baseline --no-boundary --no-setup" ;;
    c5q) echo "$C5 --steps 8 --warmup 3 --no-boundary --no-cpu-baseline --no-setup" ;;
  esac
}
case $PART in
ab)
  # A/B of library variants: VARIANTS="- name ..." (eraytracer_amd/variants/librtmi355x_NAME.so; - = default)
  : > gpurun_out/${TAG}_ab.txt
  for rep in $(seq 1 ${REPS:-2}); do
    for c in ${CFGS:-c3dq c5q}; do
      for v in ${VARIANTS:--}; do
        lib=""; [ "$v" = "-" ] || lib="eraytracer_amd/variants/librtmi355x_$v.so"
        RT_LIB_PATH=$lib timeout -k 10 300 python bench.py $(cfg_args $c) > gpurun_out/${TAG}_ab_one.json 2> gpurun_out/${TAG}_ab_one.err \
          || { tail -5 gpurun_out/${TAG}_ab_one.err; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline',{}); print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame', 'dom', r.get('launch_ms_live'))" gpurun_out/${TAG}_ab_one.json "$c $v rep$rep" | tee -a gpurun_out/${TAG}_ab.txt || exit 1
      done
    done
  done ;;
envab)
  # A/B of run-time knobs: ENVS="- RT_BVH_LEVEL=3 ..." (each item one VAR=value, or - for none)
  : > gpurun_out/${TAG}_envab.txt
  for rep in $(seq 1 ${REPS:-2}); do
    for c in ${CFGS:-c3dq c5q}; do
      for e in ${ENVS:--}; do
        ev=""; [ "$e" = "-" ] || ev="$e"
        env $ev timeout -k 10 300 python bench.py $(cfg_args $c) > gpurun_out/${TAG}_envab_one.json 2> gpurun_out/${TAG}_envab_one.err \
          || { tail -5 gpurun_out/${TAG}_envab_one.err; exit 1; }
        python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d.get('roofline',{}); print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame', 'dom', r.get('launch_ms_live'))" gpurun_out/${TAG}_envab_one.json "$c $e rep$rep" | tee -a gpurun_out/${TAG}_envab.txt || exit 1
      done
    done
  done ;;
lim)
  make -C oracle > /dev/null || exit 1
  timeout -k 10 900 python -u -m pytest tests/test_gpu_limits.py -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/pytest_lim_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_lim_$TAG.log; exit 1; }
  grep -E "PASS|FAIL|depth|passed|failed" gpurun_out/pytest_lim_$TAG.log | tail -20 ;;
test)
  make -C oracle > /dev/null || exit 1
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || { tail -5 gpurun_out/smoke_$TAG.log; exit 1; }
  tail -1 gpurun_out/smoke_$TAG.log
  bash scripts/debug_lists.sh run > gpurun_out/debug_lists_$TAG.log 2>&1 || { tail -30 gpurun_out/debug_lists_$TAG.log; exit 1; }
  tail -1 gpurun_out/debug_lists_$TAG.log ;;
c3)
  b c3d --steps 20 --warmup 5 --no-boundary --no-cpu-baseline || exit 1 ;;
setup)
  b c3d --steps 20 --warmup 5 --no-boundary --no-cpu-baseline || exit 1
  b c3d_q8 --steps 20 --warmup 5 --no-boundary --no-cpu-baseline --hw-queues 8 --no-setup || exit 1
  b c5s $C5 --steps 6 --warmup 3 --no-boundary --no-cpu-baseline || exit 1
  timeout -k 10 300 python scripts/n8_floor.py > gpurun_out/${TAG}_n8_floor.json 2> gpurun_out/${TAG}_n8_floor.err || { tail -5 gpurun_out/${TAG}_n8_floor.err; exit 1; }
  cat gpurun_out/${TAG}_n8_floor.json
  python3 -c "import json,sys; [print(n, json.dumps(json.load(open(f'gpurun_out/${TAG}_bench_'+n+'.json')).get('setup'))) for n in ('c3d','c5s')]" ;;
bench)
  make -C oracle > /dev/null || exit 1
  timeout -k 10 200 python scripts/cpu_config1.py > gpurun_out/${TAG}_cfg1.json && cat gpurun_out/${TAG}_cfg1.json || exit 1
  b c3d --steps 20 --warmup 5 --no-boundary --no-cpu-baseline || exit 1
  b c3 || exit 1
  b c2 $C2 --no-cpu-baseline || exit 1
  b c4 --size 8192 --no-cpu-baseline --no-boundary || exit 1
  b c5 $C5 --steps 10 --warmup 4 --no-boundary --cpu-seconds 10 || exit 1 ;;
prof3)
  bash scripts/profile.sh prof_${TAG}_c3 > gpurun_out/prof_${TAG}_c3.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c3.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c3 gpurun_out/${TAG}_c3_pmc.json s64-4096x4096-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_c3_pmc.txt || exit 1
  grep -E "window_ns|f64_issue|wait_any_share|hbm_bytes" gpurun_out/${TAG}_c3_pmc.txt ;;
pmcv)
  # instruction counts per kernel of library variants (VARIANTS as for ab; PMCV_ARGS: bench.py arguments)
  for v in ${VARIANTS:--}; do
    lib=""; [ "$v" = "-" ] || lib="eraytracer_amd/variants/librtmi355x_$v.so"
    RT_LIB_PATH=$lib timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_BRANCH \
      -d gpurun_out/pmcv_$TAG/$v -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --iso 0 --settle 0 --no-cpu-baseline --no-boundary --no-setup ${PMCV_ARGS:-} > gpurun_out/pmcv_${TAG}_$v.log 2>&1 || { tail -5 gpurun_out/pmcv_${TAG}_$v.log; exit 1; }
  done
  python3 scripts/pmc_variants.py gpurun_out/pmcv_$TAG > gpurun_out/pmcv_$TAG.txt || exit 1
  tail -8 gpurun_out/pmcv_$TAG.txt
  rm -rf gpurun_out/pmcv_$TAG ;;
prof2)
  bash scripts/profile.sh prof_${TAG}_c2 $C2 > gpurun_out/prof_${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c2.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c2 gpurun_out/${TAG}_c2_pmc.json default-1920x1080-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_c2_pmc.txt || exit 1
  grep -E "window_ns|f64_issue|wait_any_share|hbm_bytes" gpurun_out/${TAG}_c2_pmc.txt ;;
prof5)
  bash scripts/profile.sh prof_${TAG}_c5 $C5 --steps 6 --warmup 3 --iso 4 > gpurun_out/prof_${TAG}_c5.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c5.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c5 gpurun_out/${TAG}_c5_pmc.json s256-4096x4096-d8-exact-f32-n1-spp16 6 4 16 > gpurun_out/${TAG}_c5_pmc.txt || exit 1
  grep -E "window_ns|f64_issue|wait_any_share|hbm_bytes" gpurun_out/${TAG}_c5_pmc.txt ;;
esac
