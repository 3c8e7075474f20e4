# Parity of a variant library, then interleaved A/B bench runs against the default build:
#   bash scripts/gpu_ab_pair.sh TAG VARIANT_LIB ROUNDS "label:bench args" ...
set -o pipefail
TAG=$1; VLIB=$2; ROUNDS=$3; shift 3
mkdir -p gpurun_out
make -C oracle > /dev/null
RT_LIB_PATH=$PWD/$VLIB timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_$TAG.log | head -20; tail -3 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
for r in $(seq 1 $ROUNDS); do
for spec in "$@"; do
  label=${spec%%:*}; args=${spec#*:}
  for v in base var; do
    if [ $v = var ]; then export RT_LIB_PATH=$PWD/$VLIB; else unset RT_LIB_PATH; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $args > gpurun_out/ab_${TAG}.json 2> gpurun_out/ab_${TAG}.err || { echo "$label $v failed"; tail -5 gpurun_out/ab_${TAG}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame')" gpurun_out/ab_${TAG}.json $label $v
  done
done
done
