#!/bin/bash
# Extra PMC passes (LDS conflicts / waits, instruction and scalar caches) over a bench run.
#   bash scripts/pmc_extra.sh TAG [bench args]   (on the GPU box; one rocprofv3 run per counter set)
set -o pipefail
TAG=${1:-pmcx}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --steps 20 --warmup 10 --iso 20 --settle 0 --no-cpu-baseline --no-boundary --no-setup $*"
i=0
for P in "SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_LDS_UNALIGNED_STALL SQ_INST_LEVEL_LDS" \
         "SQC_DCACHE_MISSES SQC_ICACHE_MISSES SQ_IFETCH SQ_INST_LEVEL_SMEM SQ_INST_LEVEL_VMEM SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P -d $OUT/pmc$i -o run --output-format csv -- python3 $BENCH > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i failed: $P"; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, glob, re, sys, collections
out = sys.argv[1]
tot = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.defaultdict(int)
for f in glob.glob(out + "/pmc*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        m = re.search(r"(k_\w+)(<[^>]*>)?", r["Kernel_Name"])
        k = m.group(0)[:60] if m else r["Kernel_Name"][:40]
        tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
for k, c in sorted(tot.items()):
    print(k)
    for n, v in sorted(c.items()):
        print(f"   {n:28s} {v:16.4g}")
PY
