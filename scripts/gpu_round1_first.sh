set -o pipefail
mkdir -p gpurun_out
which erl > gpurun_out/which_erl.txt 2>&1 || echo "no erl" > gpurun_out/which_erl.txt
nproc > gpurun_out/nproc.txt; lscpu > gpurun_out/lscpu.txt 2>&1 || true
make -C oracle > /dev/null
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu 2>&1 | tee gpurun_out/pytest_gpu1.log
