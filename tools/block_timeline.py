"""Per-kernel busy time of the last layer's block loop (after the Cholesky) from a rocprofv3
kernel trace of bench.py (dev tool): python tools/block_timeline.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nm = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:45]
i0 = [i for i, r in enumerate(rows) if "copy_upper" in r["Kernel_Name"]][-1]
st = [k for k in range(i0, len(rows)) if "ssr_" in rows[k]["Kernel_Name"] or "transpose" in rows[k]["Kernel_Name"]][0]
nx = [k for k in range(st, len(rows)) if "gram16" in rows[k]["Kernel_Name"]]
en = nx[0] if nx else len(rows)
busy, cnt = defaultdict(float), defaultdict(int)
gap, last = 0.0, int(rows[st]["Start_Timestamp"])
for r in rows[st:en]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap += max(0, s - last) / 1e3
    last = max(last, e)
    busy[nm(r)] += (e - s) / 1e3
    cnt[nm(r)] += 1
print(f"block phase span {(last - int(rows[st]['Start_Timestamp'])) / 1e3:.1f} us, gaps {gap:.1f} us")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {v:8.1f} us {cnt[k]:4d}x avg {v / cnt[k]:6.2f}  {k}")
