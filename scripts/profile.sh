# usage (on the GPU box): bash scripts/profile.sh TAG [bench args]
# rocprofv3 kernel-trace stats + separate PMC passes (counters never combined with tracing domains).
set -o pipefail
TAG=${1:-prof}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 10 --iso 20 --settle 0 --no-cpu-baseline --no-boundary --no-setup $*"
timeout -k 10 120 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 $BENCH > $OUT/trace.log 2>&1 || exit 1
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS GRBM_GUI_ACTIVE" \
         "SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
         "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_CVT" \
         "FETCH_SIZE" "WRITE_SIZE" \
         "SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT64 SQ_INSTS_BRANCH SQ_INSTS_LDS_LOAD SQ_INSTS_SMEM_NORM"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $OUT/pmc$i -o run --output-format csv -- python3 $BENCH > $OUT/pmc$i.log 2>&1 || echo "pmc pass $i failed: $P" >> $OUT/failed.txt
done
ls -R $OUT | head -50
