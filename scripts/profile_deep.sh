# Latency / cache counters per kernel (one rocprofv3 --pmc pass per group):
#   bash scripts/profile_deep.sh TAG [bench args]
set -o pipefail
TAG=${1:-deep}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 10 --warmup 4 --iso 10 --settle 0 --no-cpu-baseline --no-boundary $*"
i=0
for P in "SQ_INSTS_SMEM SQ_INST_LEVEL_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INST_LEVEL_VMEM SQ_INSTS_LDS SQ_INST_LEVEL_LDS SQ_WAVE_CYCLES" \
         "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ SQC_TC_STALL" \
         "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
         "TCC_HIT_sum TCC_MISS_sum" \
         "SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM SQ_WAVES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/pmc$i -o run --output-format csv -- python3 $BENCH > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed: $P" >> $OUT/failed.txt
done
cat $OUT/failed.txt 2>/dev/null
python3 scripts/deep_summary.py $OUT
