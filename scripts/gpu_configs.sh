# BASELINE.json configs on one MI355X (config 4's 2/4/8-GPU legs are the driver's): one bench line each.
set -o pipefail
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 120 python scripts/cpu_config1.py > gpurun_out/cfg1.json || exit 1
cat gpurun_out/cfg1.json
b() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/cfg_$name.json 2> gpurun_out/cfg_$name.err || { tail -5 gpurun_out/cfg_$name.err; exit 1; }; cat gpurun_out/cfg_$name.json; }
b c2 --scene default --width 1920 --height 1080 --depth 5 && \
b c3 && \
b c4 --size 8192 --no-cpu-baseline && \
b c5 --scene s256 --depth 8 --spp 16 --steps 10 --warmup 4 --no-boundary
