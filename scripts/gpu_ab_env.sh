# A/B of environment switches on the default bench (no boundary / CPU legs):
#   bash scripts/gpu_ab_env.sh "ENV=a" "ENV=b" ...   ("-" = no extra environment)
set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/ab.jsonl
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  env $v timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $BENCH_ARGS > gpurun_out/ab_one.json 2> gpurun_out/ab_one.err || { tail -5 gpurun_out/ab_one.err; exit 1; }
  python3 -c "
import json,sys; d=json.load(open('gpurun_out/ab_one.json')); r=d['roofline']
print(json.dumps({'env': sys.argv[1], 'value': d['value'], 'ms': d['ms_per_step'], 'dom_ms': r.get('launch_ms_live'), 'frac': r.get('frac')}))" "$v" | tee -a gpurun_out/ab.jsonl
done
