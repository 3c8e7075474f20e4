# Bench lines of BASELINE configs 2-5 (config 3 with the CPU-baseline and boundary legs):
#   bash scripts/gpu_bench_lines.sh TAG
set -o pipefail
TAG=${1:-bl}
mkdir -p gpurun_out
b() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_bench_$name.json 2> gpurun_out/${TAG}_bench_$name.err || { tail -5 gpurun_out/${TAG}_bench_$name.err; exit 1; }; python3 -c "import json,sys; d=json.load(open(sys.argv[1])); r=d['roofline']; print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame; frac', r.get('frac'), 'valu', r.get('valu_issue_frac'), r.get('profile'))" gpurun_out/${TAG}_bench_$name.json $name; }
C2="--scene default --width 1920 --height 1080 --depth 5"
C5="--scene s256 --depth 8 --spp 16"
b c3 && b c2 $C2 --no-cpu-baseline && b c4 --size 8192 --no-cpu-baseline --no-boundary && b c5 $C5 --steps 10 --warmup 4 --no-boundary --cpu-seconds 10
