set -o pipefail
export GPU_MAX_HW_QUEUES=8
timeout -k 10 120 python scripts/fr_overlap.py 4 && timeout -k 10 120 python scripts/fr_overlap.py 4 lv && \
timeout -k 10 120 env RT_LIT_STREAM=0 python scripts/frame_overlap.py --reps 40 --inflight 4
