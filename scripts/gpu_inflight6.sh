set -o pipefail
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary "$@" > gpurun_out/b4.json 2> gpurun_out/b4.err || { tail -20 gpurun_out/b4.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/b4.json'));print('$*', d['value'], d['ms_per_step'], d['kernel_ms'], d['config']['inflight'])"; }
export GPU_MAX_HW_QUEUES=8
timeout -k 10 120 python scripts/fr_overlap.py 4
b
b --steps 400 --warmup 400
timeout -k 10 120 python scripts/fr_overlap.py 4
