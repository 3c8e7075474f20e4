# Bench lines + profiles of BASELINE configs 2 and 5 on one MI355X: bash scripts/gpu_c25.sh TAG
set -o pipefail
TAG=${1:-c25}
mkdir -p gpurun_out
make -C oracle > /dev/null
b() { name=$1; shift; timeout -k 10 600 python bench.py "$@" > gpurun_out/${TAG}_$name.json 2> gpurun_out/${TAG}_$name.err || { tail -5 gpurun_out/${TAG}_$name.err; exit 1; }; cat gpurun_out/${TAG}_$name.json; }
b c2 --scene default --width 1920 --height 1080 --depth 5 --no-cpu-baseline && \
b c5 --scene s256 --depth 8 --spp 16 --steps 10 --warmup 4 --no-boundary --no-cpu-baseline && \
bash scripts/gpu_configs_profile.sh $TAG
