# A/B benches with env vars: bash scripts/gpu_ab2.sh TAG "label|ENV=val ...|bench args" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { tail -40 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for spec in "$@"; do
  IFS='|' read -r label envs args <<< "$spec"
  env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-boundary $args > gpurun_out/ab_${TAG}_$label.json 2>gpurun_out/ab_${TAG}_$label.err || { echo "$label failed"; tail -5 gpurun_out/ab_${TAG}_$label.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_$label.json')); print('$label', d['value'], 'Mpx/s kernel_ms', d['kernel_ms'], 'ms_step', d['ms_per_step'])"
done
