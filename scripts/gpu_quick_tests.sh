# Quick GPU correctness subset then an env A/B: bash scripts/gpu_quick_tests.sh "ENV=a" ...
set -o pipefail
make -C oracle > /dev/null
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/quick.log 2>&1 || { tail -30 gpurun_out/quick.log; exit 1; }
tail -1 gpurun_out/quick.log
bash scripts/gpu_ab_env.sh "$@"
