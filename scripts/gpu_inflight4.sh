set -o pipefail
b() { timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary "$@" > gpurun_out/b4.json 2> gpurun_out/b4.err || { tail -20 gpurun_out/b4.err; exit 1; }; python -c "import json;d=json.load(open('gpurun_out/b4.json'));print('$*', d['value'], d['ms_per_step'], d['kernel_ms'], d['config']['inflight'])"; }
b --steps 40 --warmup 8
b --steps 100 --warmup 60
b --steps 200 --warmup 200
b --steps 100 --warmup 60 --inflight 1
b --steps 100 --warmup 60 --inflight 3
