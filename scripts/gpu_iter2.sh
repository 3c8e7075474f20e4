# Iteration check: GPU parity suite (optionally a subset), then bench lines of the given configs.
#   bash scripts/gpu_iter2.sh TAG "pytest selector or empty" "label:bench args" ...
set -o pipefail
TAG=$1; SEL=${2:-tests}; shift 2
mkdir -p gpurun_out
make -C oracle > /dev/null
if [ "$SEL" != "none" ]; then
timeout -k 10 900 python -u -m pytest $SEL -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { grep -E "FAIL|Error|assert" gpurun_out/pytest_$TAG.log | head -30; tail -5 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
fi
for spec in "$@"; do
  label=${spec%%:*}; args=${spec#*:}
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $args > gpurun_out/it_${TAG}_$label.json 2> gpurun_out/it_${TAG}_$label.err || { echo "$label failed"; tail -5 gpurun_out/it_${TAG}_$label.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame; dominant', r.get('kernel'), r.get('launch_ms_live'), 'ms')" gpurun_out/it_${TAG}_$label.json $label
done
