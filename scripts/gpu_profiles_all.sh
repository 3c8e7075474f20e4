set -o pipefail
TAG=${1:-r02}
mkdir -p gpurun_out
make -C oracle > /dev/null
bash scripts/profile.sh prof_${TAG}_c3 > gpurun_out/prof_${TAG}_c3.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c3.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c3 gpurun_out/${TAG}_c3_pmc.json s64-4096x4096-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_c3_pmc.txt
tail -16 gpurun_out/${TAG}_c3_pmc.txt
bash scripts/gpu_configs_profile.sh $TAG
