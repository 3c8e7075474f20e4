#!/bin/bash
# PC sampling (host trap, time-based) of the config-3 bench; summary by scripts/pcs_summary.py
set -o pipefail
mkdir -p gpurun_out/pcs
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/pcs/list.txt 2>&1; grep -i -A3 "pc_sampling\|pc sampling" gpurun_out/pcs/list.txt | head -20
timeout -s KILL 200 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 1 -d gpurun_out/pcs -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 \
    --iso 0 --settle 0 --no-cpu-baseline --no-boundary > gpurun_out/pcs/log.txt 2>&1; echo "pcs rc=$?"
tail -5 gpurun_out/pcs/log.txt; ls -la gpurun_out/pcs | head
