# Round evidence on the GPU box: bash scripts/gpu_round_profile.sh TAG [nobench]
#   GPU parity suite, the default bench line (with CPU baseline), a rocprofv3 kernel trace
#   (--kernel-trace --stats) of the bench and separate PMC passes, summarised per frame.
set -o pipefail
TAG=${1:-round}
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 900 python -u -m pytest tests -x -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1 || { tail -30 gpurun_out/pytest_$TAG.log; exit 1; }
tail -1 gpurun_out/pytest_$TAG.log
timeout -k 10 600 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || { tail -20 gpurun_out/bench_$TAG.err; exit 1; }
cat gpurun_out/bench_$TAG.json
bash scripts/profile.sh prof_$TAG > gpurun_out/prof_$TAG.log 2>&1 || { tail -20 gpurun_out/prof_$TAG.log; exit 1; }
python3 scripts/pmc_summary.py gpurun_out/prof_$TAG gpurun_out/${TAG}_pmc.json s64-4096x4096-d5-exact-f32-n1 20 20 > gpurun_out/${TAG}_pmc.txt
tail -25 gpurun_out/${TAG}_pmc.txt
