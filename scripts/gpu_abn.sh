# Interleaved A/B bench runs of several library variants (no test run):
#   bash scripts/gpu_abn.sh TAG ROUNDS "bench args" LIB...   (LIB "-" = the default build)
set -o pipefail
TAG=$1; ROUNDS=$2; ARGS=$3; shift 3
mkdir -p gpurun_out
for r in $(seq 1 $ROUNDS); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset RT_LIB_PATH; else export RT_LIB_PATH=$PWD/$lib; fi
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $ARGS > gpurun_out/abn_${TAG}.json 2> gpurun_out/abn_${TAG}.err || { echo "$lib failed"; tail -5 gpurun_out/abn_${TAG}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame')" gpurun_out/abn_${TAG}.json $(basename $lib)
  done
done
