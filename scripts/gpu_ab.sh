# A/B benches on the GPU box: bash scripts/gpu_ab.sh TAG "label:libpath:args" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; args=${rest#*:}
  if [ -n "$lib" ]; then export RT_LIB_PATH=$lib; else unset RT_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-boundary $args > gpurun_out/ab_${TAG}_$label.json 2>gpurun_out/ab_${TAG}_$label.err || { echo "$label failed"; tail -5 gpurun_out/ab_${TAG}_$label.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_${TAG}_$label.json')); print('$label', d['value'], 'Mpx/s kernel_ms', d['kernel_ms'], 'valu_frac', d['roofline']['frac'])"
done
