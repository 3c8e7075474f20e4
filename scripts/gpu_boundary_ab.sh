set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/bab.jsonl
for v in "RT_BAND_MB=24" "RT_BAND_MB=48" "RT_BAND_MB=96" "RT_BAND_MB=1000" "RT_BAND_MB=24 RT_CTX_SIDE_STREAMS=1" "RT_BAND_MB=48 RT_COPY_STREAMS=2"; do
  env $v timeout -k 10 120 python scripts/boundary_ab.py >> gpurun_out/bab.jsonl || exit 1
done
cat gpurun_out/bab.jsonl
