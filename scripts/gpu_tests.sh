# GPU test suite on the box: bash scripts/gpu_tests.sh TAG [pytest selectors...]
set -o pipefail
TAG=${1:-t}; shift || true
mkdir -p gpurun_out
make -C oracle > /dev/null
SEL=${*:-tests}
timeout -k 10 1000 python -u -m pytest $SEL -x -v -s -m gpu --timeout 600 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|pixels not bit|first .* ms|passed|failed" gpurun_out/pytest_$TAG.log | tail -60
exit $rc
