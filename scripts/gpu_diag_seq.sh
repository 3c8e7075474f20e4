set -o pipefail
mkdir -p gpurun_out/diag
export TMPDIR=/tmp
make -C oracle > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/diag/trace -o run --output-format csv -- python3 -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_fullsize.py -x -q -m gpu -k "not fused_wavefront and not general_pow and not repeated_render" > gpurun_out/diag/pytest.log 2>&1
echo "rc=$?"
tail -5 gpurun_out/diag/pytest.log
f=$(ls gpurun_out/diag/trace/*/*kernel_trace.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find gpurun_out/diag/trace -name "*kernel_trace.csv" | head -1)
echo "$f"
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Dispatch_Id"]))
print(len(rows), "dispatches")
for r in rows[-25:]:
    print(r["Dispatch_Id"], r["Kernel_Name"][:110], r.get("Grid_Size", ""), r.get("Workgroup_Size", ""))
PY
