set -o pipefail
make -C oracle > /dev/null
RT_ENGINE=wave timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_wf4.log 2>&1 || { tail -30 gpurun_out/pytest_wf4.log; exit 1; }
tail -1 gpurun_out/pytest_wf4.log
bash scripts/gpu_ab2.sh wf4 "wave|RT_ENGINE=wave|" "mega|RT_ENGINE=mega|" "wave_def|RT_ENGINE=wave|--scene default --size 1920" "wave256|RT_ENGINE=wave|--scene s256 --depth 8" && bash scripts/ktrace.sh s64c RT_ENGINE=wave --
