# A/B benches without the test suite, interleaved twice: bash scripts/gpu_ab3.sh TAG "label|ENV=val ...|bench args" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for round in 1 2; do
for spec in "$@"; do
  IFS='|' read -r label envs args <<< "$spec"
  env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $args > gpurun_out/ab_${TAG}_$label.json 2>gpurun_out/ab_${TAG}_$label.err || { echo "$label failed"; tail -5 gpurun_out/ab_${TAG}_$label.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_$label.json')); print('$label', d['value'], 'Mpx/s ms_step', d['ms_per_step'])"
done
done
