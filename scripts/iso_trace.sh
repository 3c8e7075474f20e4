#!/bin/bash
# Per-kernel durations of frames rendered alone (bench.py --iso: the last ISO frames, one at a time
# on one context): rocprofv3 kernel trace, summarised by scripts/iso_summary.py.
#   bash scripts/iso_trace.sh TAG [ENV=VALUE ...] -- [bench args]
set -o pipefail
TAG=$1; shift
ENVS=""; while [ "$1" != "--" ] && [ -n "$1" ]; do ENVS="$ENVS $1"; shift; done; shift
OUT=gpurun_out/iso_$TAG
mkdir -p $OUT; export TMPDIR=/tmp
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT -o run --output-format csv -- python3 bench.py \
    --steps 10 --warmup 5 --iso 20 --settle 0.2 --no-cpu-baseline --no-boundary "$@" > $OUT/log.txt 2>&1 || { tail $OUT/log.txt; exit 1; }
python3 scripts/iso_summary.py $OUT 20
