#!/bin/bash
# Round 3: producer-built lists — list tests, bench lines (configs 3, 5), then the whole suite.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_frames.py -k "fused_path or brute" -v -s --timeout 250 \
    --timeout-method thread > gpurun_out/r03_lists.log 2>&1; echo "lists rc=$?"
timeout -k 10 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline --no-boundary > gpurun_out/r03_bench_c3.json 2> gpurun_out/r03_bench_c3.err &&
cut -c1-300 gpurun_out/r03_bench_c3.json &&
timeout -k 10 300 python bench.py --scene s256 --depth 8 --spp 16 --steps 6 --warmup 2 --iso 3 --no-cpu-baseline --no-boundary > gpurun_out/r03_bench_c5.json 2> gpurun_out/r03_bench_c5.err &&
cut -c1-300 gpurun_out/r03_bench_c5.json &&
RT_FUSE_SHADE=0 timeout -k 10 300 python bench.py --steps 50 --warmup 20 --no-cpu-baseline --no-boundary > gpurun_out/r03_bench_c3_nofuse.json 2> gpurun_out/r03_bench_c3_nofuse.err &&
cut -c1-300 gpurun_out/r03_bench_c3_nofuse.json
