# Profiles (kernel trace + PMC) and bench lines of BASELINE configs 2 and 5 on one MI355X:
#   bash scripts/gpu_configs_profile.sh TAG
set -o pipefail
TAG=${1:-cfg}
mkdir -p gpurun_out
make -C oracle > /dev/null
C2="--scene default --width 1920 --height 1080 --depth 5"
C5="--scene s256 --depth 8 --spp 16"
bash scripts/profile.sh prof_${TAG}_c2 $C2 > gpurun_out/prof_${TAG}_c2.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c2.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c2 gpurun_out/${TAG}_c2_pmc.json default-1920x1080-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_c2_pmc.txt
tail -6 gpurun_out/${TAG}_c2_pmc.txt
bash scripts/profile.sh prof_${TAG}_c5 $C5 --steps 6 --warmup 3 --iso 4 > gpurun_out/prof_${TAG}_c5.log 2>&1 || { tail -20 gpurun_out/prof_${TAG}_c5.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_${TAG}_c5 gpurun_out/${TAG}_c5_pmc.json s256-4096x4096-d8-exact-f32-n1-spp16 6 4 16 > gpurun_out/${TAG}_c5_pmc.txt
tail -16 gpurun_out/${TAG}_c5_pmc.txt
