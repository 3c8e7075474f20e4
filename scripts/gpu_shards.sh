set -o pipefail
timeout -k 10 120 env RT_LIT_STREAM=1 python scripts/shard_render_time.py && \
timeout -k 10 120 env RT_LIT_STREAM=0 python scripts/shard_render_time.py && \
timeout -k 10 120 env RT_LIT_STREAM=1 GPU_MAX_HW_QUEUES=8 python scripts/shard_render_time.py
