set -o pipefail
for sc in s4 s8 s16 s24; do
  BENCH_ARGS="--scene $sc --steps 40 --warmup 20" bash scripts/gpu_ab_env.sh RT_ENGINE=fused RT_ENGINE=wave | sed "s/^/$sc /" || exit 1
done
