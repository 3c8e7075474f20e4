set -o pipefail
OUT=gpurun_out/pcs
mkdir -p $OUT
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 1 -d $OUT -o run --output-format csv -- python3 bench.py --steps 10 --warmup 2 --iso 10 --settle 0 --no-cpu-baseline --no-boundary > $OUT/log.txt 2>&1
echo "rc=$?"
tail -5 $OUT/log.txt
ls -la $OUT $OUT/* | head -30
