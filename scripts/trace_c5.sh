# Kernel trace of config 5 (per-kernel durations per sample pass): bash scripts/trace_c5.sh TAG [env...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
env "$@" timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --scene s256 --depth 8 --spp 16 --steps 6 --warmup 3 --iso 4 --settle 0 --no-cpu-baseline --no-boundary > $OUT/trace.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $OUT $OUT/summary.json s256-4096x4096-d8-exact-f32-n1-spp16 6 4 16 | grep -E "us \(alone|window"
