"""Summarise a rocprofv3 kernel trace: per-kernel busy time and the idle gaps of the last
`--last` dispatches window.  usage: python tools/timeline.py run_kernel_trace.csv [first_kernel_substr]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
start_key = sys.argv[2] if len(sys.argv) > 2 else None
if start_key:
    idx = [i for i, r in enumerate(rows) if start_key in r["Kernel_Name"]]
    rows = rows[idx[-1]:] if idx else rows
t0 = int(rows[0]["Start_Timestamp"])
t1 = max(int(r["End_Timestamp"]) for r in rows)
busy = defaultdict(float)
cnt = defaultdict(int)
cover = 0
last_end = t0
for r in rows:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:70]
    busy[name] += (e - s) / 1e3
    cnt[name] += 1
    if e > last_end:
        cover += e - max(s, last_end)
        last_end = e
span = (t1 - t0) / 1e3
print(f"window {span:.1f} us, covered by kernels {cover / 1e3:.1f} us ({100 * cover / 1e3 / span:.0f}%), {len(rows)} dispatches")
for k, v in sorted(busy.items(), key=lambda x: -x[1])[:12]:
    print(f"  {v:9.1f} us  {cnt[k]:5d}x  {k}")
