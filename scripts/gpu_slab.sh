# Compact-gather checks on the GPU box: codec timing at N = 2/4/8 shard geometry.
set -o pipefail
mkdir -p gpurun_out
for ns in 2 4 8; do
  timeout -k 10 120 python scripts/slab_codec_bench.py --ns $ns || exit 1
done
