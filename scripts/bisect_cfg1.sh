# temporary (round 4): config-1 parity test against library builds of earlier commits
make -C oracle > /dev/null || exit 1
for v in at_bb84211 at_39546d3 at_7a588f1 at_c6caee0 -; do
  lib=""; [ "$v" = "-" ] || lib=eraytracer_amd/variants/librtmi355x_$v.so
  RT_LIB_PATH=$lib timeout -k 10 120 python -m pytest tests/test_gpu_fullsize.py -x -q -m gpu -k "config1 or config2" 2>&1 | grep -E "not bit-identical|passed|failed" | sed "s/^/$v: /" | head -4
done
