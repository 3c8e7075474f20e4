# Config 5 per-level kernel times under different RT_BVH_LEVEL settings: bash scripts/gpu_c5_levels.sh TAG LEVEL...
set -o pipefail
TAG=$1; shift
mkdir -p gpurun_out; export TMPDIR=/tmp
for L in "$@"; do
  RT_BVH_LEVEL=$L timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kt_${TAG}_$L -o run --output-format csv -- python3 bench.py --scene s256 --depth 8 --spp 16 --steps 3 --warmup 1 --settle 0 --no-cpu-baseline --no-boundary > gpurun_out/kt_${TAG}_$L.log 2>&1 || { tail gpurun_out/kt_${TAG}_$L.log; exit 1; }
  echo "== RT_BVH_LEVEL=$L $(tail -1 gpurun_out/kt_${TAG}_$L.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], "ms/frame")')"
  python3 scripts/klevels.py gpurun_out/kt_${TAG}_$L | head -30
done
