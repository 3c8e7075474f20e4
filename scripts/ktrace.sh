# per-kernel time split (rocprofv3 kernel trace) for one bench configuration: bash scripts/ktrace.sh TAG [ENV=..] -- bench args
set -o pipefail
TAG=$1; shift
ENVS=""; while [ "$1" != "--" ] && [ -n "$1" ]; do ENVS="$ENVS $1"; shift; done; shift
mkdir -p gpurun_out; export TMPDIR=/tmp
env $ENVS timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/kt_$TAG -o run --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-boundary "$@" > gpurun_out/kt_$TAG.log 2>&1 || { tail gpurun_out/kt_$TAG.log; exit 1; }
python3 - gpurun_out/kt_$TAG <<'PY'
import csv, glob, sys, re
f = glob.glob(sys.argv[1] + "/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    n = r["Name"]
    if "k_" not in n: continue
    short = re.sub(r"\(rtl::.*|\(.*", "", n.replace("void (anonymous namespace)::", ""))
    print(f"{short:45s} calls={r['Calls']:>4} avg_us={float(r['AverageNs'])/1e3:9.1f} total_ms={float(r['TotalDurationNs'])/1e6:8.2f}")
PY
