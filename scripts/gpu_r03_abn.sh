#!/bin/bash
# A/B of several variant libraries (eraytracer_amd/variants/librtmi355x_<name>.so; "cur" = the
# in-tree build): brute-force parity of each variant, then alternating bench lines of config 3
# (and config 5 with C5=1).
#   bash scripts/gpu_r03_abn.sh cur beam ...
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
lib() { if [ "$1" = cur ]; then echo ""; else echo "RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_$1.so"; fi; }
for v in "$@"; do
  [ "$v" = cur ] && continue
  [ "${PARITY_K:-brute}" = none ] && continue
  timeout -k 10 300 env $(lib $v) python -u -m pytest ${PARITY_FILES:-tests/test_gpu_frames.py} -k "${PARITY_K:-brute}" -q \
      --timeout 250 --timeout-method thread > gpurun_out/abn_parity_$v.log 2>&1 || { echo "PARITY FAIL $v"; tail -5 gpurun_out/abn_parity_$v.log; exit 1; }
  echo "parity ok $v"
done
for rep in $(seq 1 ${REPS:-2}); do
  [ "${C3:-1}" = 1 ] || break
  for v in "$@"; do
    timeout -k 10 200 env $(lib $v) python bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-boundary > gpurun_out/abn_c3_$v.json 2>/dev/null || exit 1
    echo "c3 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abn_c3_$v.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('launch_ms_live'))")"
  done
done
if [ "${C2:-0}" = 1 ]; then
  for rep in $(seq 1 ${REPS:-2}); do
  for v in "$@"; do
    timeout -k 10 200 env $(lib $v) python bench.py --scene default --size 0 --width 1920 --height 1080 --steps 200 --warmup 50 --no-cpu-baseline --no-boundary > gpurun_out/abn_c2_$v.json 2>/dev/null || exit 1
    echo "c2 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abn_c2_$v.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('launch_ms_live'))")"
  done
  done
fi
if [ "${C5:-0}" = 1 ]; then
  for v in "$@"; do
    timeout -k 10 300 env $(lib $v) python bench.py --scene s256 --depth 8 --spp 16 --steps 8 --warmup 2 --iso 3 --no-cpu-baseline --no-boundary > gpurun_out/abn_c5_$v.json 2>/dev/null || exit 1
    echo "c5 $v $(python3 -c "import json;d=json.load(open('gpurun_out/abn_c5_$v.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('launch_ms_live'))")"
  done
fi
