set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_if.log 2>&1 || { tail -30 gpurun_out/pytest_if.log; exit 1; }
tail -1 gpurun_out/pytest_if.log
for a in "" "--inflight 1" "--inflight 3" "--inflight 6"; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-boundary $a > gpurun_out/bench_if.json 2> gpurun_out/bench_if.err || { tail -20 gpurun_out/bench_if.err; exit 1; }
python -c "import json;d=json.load(open('gpurun_out/bench_if.json'));print('$a', d['value'], d['ms_per_step'], d['kernel_ms'], d['config']['inflight'])"
done
