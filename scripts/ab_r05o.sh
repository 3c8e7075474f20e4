#!/bin/bash
# Round-5 A/B batch: deferred sphere ids (lid), mixed-scene occupancy (lidmix), k_walk list prefetch (walkpf)
set -o pipefail
M="--width 1536 --height 1024 --depth 5 --no-cpu-baseline --no-boundary"
REPS=3 BENCH_CFGS="c3q c5q c2" bash scripts/gpu_r04.sh r05o ab base lid lidmix || exit 1
: > gpurun_out/r05o_mixed.txt
for rep in 1 2 3; do for v in base lid lidmix; do for sc in mixed mixed_int; do
  RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_$v.so timeout -k 10 300 python bench.py --scene $sc $M > gpurun_out/r05o_mx.json 2>gpurun_out/r05o_mx.err || { tail -5 gpurun_out/r05o_mx.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Mpx/s', d['ms_per_step'], 'ms/frame', d['config']['engine'])" gpurun_out/r05o_mx.json "$sc $v rep$rep" | tee -a gpurun_out/r05o_mixed.txt
done; done; done
RT_LIB_PATH=eraytracer_amd/variants/librtmi355x_lidmix.so timeout -k 10 600 python -u -m pytest tests/test_gpu_frames.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/r05o_pytest.log 2>&1 || { tail -30 gpurun_out/r05o_pytest.log; exit 1; }; tail -2 gpurun_out/r05o_pytest.log
REPS=3 BENCH_CFGS="c3q c5q" bash scripts/gpu_r04.sh r05p ab lidmix walkpf
REPS=2 BENCH_CFGS="c3q c5q" bash scripts/gpu_r04.sh r05q ab walkpf l1g2560 l1g5120
