#!/bin/bash
# Round 3: the whole -m gpu suite, a config-3 bench line, then a PC-sampling attempt on config 3.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 500 --timeout-method thread \
    > gpurun_out/r03_suite.log 2>&1 && echo "suite ok" && tail -3 gpurun_out/r03_suite.log &&
timeout -k 10 300 python bench.py --steps 50 --warmup 20 --cpu-seconds 10 > gpurun_out/r03_bench_c3.json 2> gpurun_out/r03_bench_c3.err &&
cat gpurun_out/r03_bench_c3.json | cut -c1-600 &&
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" &&
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time \
    --pc-sampling-interval 1 -d gpurun_out/pcs -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 \
    --iso 0 --settle 0 --no-cpu-baseline --no-boundary > gpurun_out/pcs_log.txt 2>&1; echo "pcs rc=$?"; ls -la gpurun_out/pcs 2>/dev/null | head
