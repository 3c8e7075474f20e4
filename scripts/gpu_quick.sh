# quick check: GPU parity suite + bench (no CPU baseline / boundary); usage: bash scripts/gpu_quick.sh TAG [bench args]
set -o pipefail
TAG=${1:-q}; shift || true
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_$TAG.log | head -30; tail -5 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary "$@" > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_$TAG.json'));print('bench', d['value'], d['ms_per_step'], d['kernel_ms'])"
done
