set -o pipefail
echo "env GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES-unset}"
b() { timeout -k 10 300 env "$@" python bench.py --steps 40 --warmup 8 --no-cpu-baseline --no-boundary > gpurun_out/b2.json 2> gpurun_out/b2.err || { tail -20 gpurun_out/b2.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/b2.json'));print('$*', d['value'], d['ms_per_step'], d['kernel_ms'], d['config']['inflight'])"; }
timeout -k 10 120 env GPU_MAX_HW_QUEUES=8 RT_LIT_STREAM=0 python scripts/frame_overlap.py --reps 40 --inflight 4 || exit 1
b GPU_MAX_HW_QUEUES=8
b GPU_MAX_HW_QUEUES=8 RT_LIT_STREAM=0
b GPU_MAX_HW_QUEUES=4
