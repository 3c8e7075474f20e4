set -o pipefail
C5="--scene s256 --depth 8 --spp 16 --steps 4 --warmup 2"
for r in 1 2; do for L in 1 2 3; do
  RT_BVH_LEVEL=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-boundary $C5 > gpurun_out/lvl.json 2> gpurun_out/lvl.err || { tail -5 gpurun_out/lvl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('level', sys.argv[2], d['value'], d['ms_per_step'])" gpurun_out/lvl.json $L
done; done
