#!/bin/bash
# Config 3 with 3..6 frames in flight (alternating, two rounds).
set -o pipefail
mkdir -p gpurun_out
for rep in 1 2; do
  for i in 4 3 5 6; do
    timeout -k 10 200 python bench.py --steps 60 --warmup 20 --inflight $i --no-cpu-baseline --no-boundary > gpurun_out/c3_if$i.json 2>/dev/null || exit 1
    echo "c3 inflight $i: $(python3 -c "import json;d=json.load(open('gpurun_out/c3_if$i.json'));print(d['value'],d['ms_per_step'])")"
  done
done
