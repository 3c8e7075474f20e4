# FETCH_SIZE / TCC read-request calibration (scripts/hbm_calib.hip; binary built on the CPU side into
# eraytracer_amd/variants/hbm_calib): bash scripts/hbm_calib.sh
set -o pipefail
OUT=gpurun_out/hbm_calib
mkdir -p $OUT
export TMPDIR=/tmp
B=eraytracer_amd/variants/hbm_calib
timeout -k 10 120 $B > $OUT/plain.txt || exit 1
timeout -s KILL 120 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $B > $OUT/trace.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/p1 -o run --output-format csv -- $B > $OUT/p1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum -d $OUT/p2 -o run --output-format csv -- $B > $OUT/p2.log 2>&1 || exit 1
cat $OUT/plain.txt
python3 - <<'PY'
import csv, glob, collections
out = collections.defaultdict(dict)
for p in ("p1", "p2"):
    for f in glob.glob(f"gpurun_out/hbm_calib/{p}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split("<")[0].split()[-1] + ("<" + r["Kernel_Name"].split("<")[1].split(">")[0] + ">" if "<" in r["Kernel_Name"] else "")
            out[k][r["Counter_Name"]] = out[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for k, v in out.items():
    print(k, {c: round(x) for c, x in v.items()})
PY
