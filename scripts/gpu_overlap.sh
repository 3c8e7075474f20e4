set -o pipefail
r() { timeout -k 10 120 env "$@" python scripts/frame_overlap.py --reps 40 --inflight $K; }
K=3 r RT_LIT_STREAM=0 && K=4 r RT_LIT_STREAM=0 && K=3 r RT_LIT_STREAM=0 GPU_MAX_HW_QUEUES=8 && K=4 r RT_LIT_STREAM=0 GPU_MAX_HW_QUEUES=8 && K=6 r RT_LIT_STREAM=0 GPU_MAX_HW_QUEUES=8
