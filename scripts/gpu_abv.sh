# A/B of library variants (no test run: ablation builds give wrong images):
#   bash scripts/gpu_abv.sh TAG "label:libpath:bench args" ...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; args=${rest#*:}
  if [ -n "$lib" ]; then export RT_LIB_PATH=$PWD/$lib; else unset RT_LIB_PATH; fi
  timeout -k 10 300 python bench.py --steps 60 --warmup 20 --no-cpu-baseline --no-boundary $args > gpurun_out/abv_${TAG}_$label.json 2>gpurun_out/abv_${TAG}_$label.err || { echo "$label failed"; tail -5 gpurun_out/abv_${TAG}_$label.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame; dominant alone', r.get('launch_ms_live'), 'ms')" gpurun_out/abv_${TAG}_$label.json $label
done
