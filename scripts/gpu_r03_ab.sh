#!/bin/bash
# A/B of the current build against a variant library: isolated-frame kernel traces + bench lines.
#   bash scripts/gpu_r03_ab.sh VARIANT [bench args]
set -o pipefail
V=$1; shift
mkdir -p gpurun_out
VL=eraytracer_amd/variants/librtmi355x_$V.so
for w in cur $V; do
  if [ $w = cur ]; then E=""; else E="RT_LIB_PATH=$VL"; fi
  timeout -k 10 200 env $E python bench.py --steps 50 --warmup 20 --no-cpu-baseline --no-boundary "$@" > gpurun_out/ab_$w.json 2> gpurun_out/ab_$w.err || exit 1
  echo "$w: $(python3 -c "import json;d=json.load(open('gpurun_out/ab_$w.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('launch_ms_live'))")"
done
bash scripts/iso_trace.sh cur -- "$@" > gpurun_out/iso_cur.txt && cat gpurun_out/iso_cur.txt &&
bash scripts/iso_trace.sh $V RT_LIB_PATH=$VL -- "$@" > gpurun_out/iso_$V.txt && cat gpurun_out/iso_$V.txt
