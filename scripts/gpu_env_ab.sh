# Interleaved A/B of an environment knob: bash scripts/gpu_env_ab.sh TAG ROUNDS "bench args" "ENV=a" "ENV=b" ...
set -o pipefail
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for e in "$@"; do
    env $e timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $ARGS > gpurun_out/env_${TAG}.json 2> gpurun_out/env_${TAG}.err || { echo "$e failed"; tail -5 gpurun_out/env_${TAG}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame')" gpurun_out/env_${TAG}.json "$e"
  done
done
