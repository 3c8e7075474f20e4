#!/bin/bash
# Config 5 variants: frames in flight and library variants (bench lines only).
#   bash scripts/gpu_r03_c5.sh "cur:4 cur:8 sparse:4 ..."   (variant:inflight)
set -o pipefail
mkdir -p gpurun_out
for vi in $1; do
  v=${vi%%:*}; i=${vi##*:}
  if [ "$v" = cur ]; then E=""; else E="RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_$v.so"; fi
  timeout -k 10 300 env $E python bench.py --scene s256 --depth 8 --spp 16 --steps 8 --warmup 2 --iso 2 --inflight $i \
      --no-cpu-baseline --no-boundary > gpurun_out/c5_${v}_$i.json 2>gpurun_out/c5_${v}_$i.err || { tail -3 gpurun_out/c5_${v}_$i.err; exit 1; }
  echo "c5 $v inflight $i: $(python3 -c "import json;d=json.load(open('gpurun_out/c5_${v}_$i.json'));print(d['value'],d['ms_per_step'],d['roofline'].get('launch_ms_live'))")"
done
