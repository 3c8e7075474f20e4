# VGPR / SGPR / scratch / occupancy per kernel of librtmi355x (compile-time, no GPU)
make -C "$(dirname "$0")/../eraytracer_amd/csrc" resource-usage 2>&1 | python3 -c '
import re, sys
cur = None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        n = m.group(1)
        d = re.search(r"(k_\w+?)I(.*?)EEv", n) or re.search(r"(k_\w+?)E", n)
        cur = (d.group(1) + ("<" + d.group(2) + ">" if d.lastindex > 1 else "")) if d else n
        print(); print(f"{cur:32s}", end="")
        continue
    for key in ("VGPRs", "TotalSGPRs", "ScratchSize", "Occupancy"):
        m = re.search(key + r": (\d+)", line)
        if m and cur:
            print(f" {key}={m.group(1)}", end="")
print()'
