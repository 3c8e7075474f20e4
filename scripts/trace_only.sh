# Kernel trace (isolated per-kernel durations) of a bench run: bash scripts/trace_only.sh TAG KEY [bench args]
set -o pipefail
TAG=$1; KEY=$2; shift 2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 --iso 20 --settle 0 --no-cpu-baseline --no-boundary "$@" > $OUT/trace.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $OUT $OUT/summary.json $KEY 20 20 $SPP | grep -E "us \(alone"
