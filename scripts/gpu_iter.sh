# One development iteration on the GPU box: the GPU test suite, then short bench lines of
# configs 3, 2 and 5 (no CPU baseline, no boundary legs).  bash scripts/gpu_iter.sh TAG [notests]
set -o pipefail
TAG=${1:-it}
mkdir -p gpurun_out
make -C oracle > /dev/null
if [ "$2" != "notests" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_$TAG.log
fi
b() { name=$1; shift; timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; exit 1; }; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame; dominant', r.get('kernel'), r.get('launch_ms_live'), 'ms')" gpurun_out/${TAG}_$name.json $name; }
b c3 && b c2 --scene default --width 1920 --height 1080 --depth 5 && b c5 --scene s256 --depth 8 --spp 16 --steps 10 --warmup 4
