# Config 5 under BVH build / staging knobs: bash scripts/gpu_sah_ab.sh ("SLACK ROWS_LDS" pairs via $CFGS)
set -o pipefail
C5="--scene s256 --depth 8 --spp 16 --steps 4 --warmup 2"
CFGS=${CFGS:-"0 1|2 1|2 0|3 1"}
for r in 1 2; do
IFS='|'; for cfg in $CFGS; do
  unset IFS; set -- $cfg
  RT_BVH_SAH_SLACK=$1 RT_BVH_ROWS_LDS=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $C5 > gpurun_out/sah.json 2> gpurun_out/sah.err || { tail -5 gpurun_out/sah.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('slack', sys.argv[2], 'rows', sys.argv[3], d['value'], d['ms_per_step'])" gpurun_out/sah.json $1 $2
  IFS='|'
done; unset IFS
done
