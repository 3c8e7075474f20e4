#!/bin/bash
# Round-4 evidence on one MI355X, in two gpurun calls (each under gpurun's 1200 s limit):
#   bash scripts/gpu_r04_evidence.sh TAG a   GPU parity suite + bench lines of configs 1-5
#   bash scripts/gpu_r04_evidence.sh TAG b   rocprofv3 kernel trace + PMC passes of configs 3, 2, 5
set -o pipefail
TAG=${1:-r04}
PART=${2:-a}
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
C2="--scene default --width 1920 --height 1080 --depth 5"
C5="--scene s256 --depth 8 --spp 16"
if [ "$PART" = a ]; then
  make -C oracle > /dev/null || exit 1
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
  b() { name=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench_$name.json 2> gpurun_out/${TAG}_bench_$name.err || { tail -5 gpurun_out/${TAG}_bench_$name.err; exit 1; }; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame')" gpurun_out/${TAG}_bench_$name.json $name; }
  timeout -k 10 200 python scripts/cpu_config1.py > gpurun_out/${TAG}_cfg1.json && cat gpurun_out/${TAG}_cfg1.json || exit 1
  b c3 || exit 1
  b c3d --steps 20 --warmup 5 --no-boundary --no-cpu-baseline || exit 1
  b c2 $C2 --no-cpu-baseline || exit 1
  b c4 --size 8192 --no-cpu-baseline --no-boundary || exit 1
  b c5 $C5 --steps 10 --warmup 4 --no-boundary --cpu-seconds 10 || exit 1
else
  bash scripts/profile.sh prof_${TAG}_c3 > gpurun_out/prof_${TAG}_c3.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c3.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c3 gpurun_out/${TAG}_c3_pmc.json s64-4096x4096-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_c3_pmc.txt || exit 1
  bash scripts/profile.sh prof_${TAG}_c2 $C2 > gpurun_out/prof_${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c2.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c2 gpurun_out/${TAG}_c2_pmc.json default-1920x1080-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_c2_pmc.txt || exit 1
  bash scripts/profile.sh prof_${TAG}_c5 $C5 --steps 6 --warmup 3 --iso 4 > gpurun_out/prof_${TAG}_c5.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c5.log; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c5 gpurun_out/${TAG}_c5_pmc.json s256-4096x4096-d8-exact-f32-n1-spp16 6 4 16 > gpurun_out/${TAG}_c5_pmc.txt || exit 1
  for c in c3 c2 c5; do echo "== $c"; grep -E "window_ns|f64_issue|wait_any_share|hbm_bytes" gpurun_out/${TAG}_${c}_pmc.txt; done
fi
