set -o pipefail
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_drv.json 2> gpurun_out/bench_drv.err || { tail -5 gpurun_out/bench_drv.err; exit 1; }
timeout -k 10 300 python bench.py > gpurun_out/bench_def.json 2> gpurun_out/bench_def.err || { tail -5 gpurun_out/bench_def.err; exit 1; }
cat gpurun_out/bench_drv.json gpurun_out/bench_def.json
