set -o pipefail
RT_FUSE_SHADE=0 timeout -k 10 120 python scripts/diag_c5.py 1 16 && \
timeout -k 10 120 python scripts/diag_c5.py 0 16 && \
timeout -k 10 120 python scripts/diag_c5.py 1 2
