set -o pipefail
mkdir -p gpurun_out
make -C oracle > /dev/null
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1
timeout -k 10 600 python bench.py --steps 10 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof1 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-boundary > gpurun_out/prof1.log 2>&1
