"""Per-iteration Cholesky timeline from a rocprofv3 kernel trace of bench.py (dev tool):
python tools/chol_timeline.py gpurun_out/trX/run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
nm = lambda r: r["Kernel_Name"].replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:40]
idx = [i for i, r in enumerate(rows) if "copy_upper" in r["Kernel_Name"]]
i0 = idx[-1]
t0 = int(rows[i0]["Start_Timestamp"])
end = [k for k in range(i0, len(rows)) if "ssr_" in rows[k]["Kernel_Name"] or "transpose" in rows[k]["Kernel_Name"]][0]
busy = defaultdict(float)
cnt = defaultdict(int)
gap = 0.0
last = int(rows[i0]["End_Timestamp"])
for r in rows[i0 + 1:end]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap += max(0, s - last) / 1e3
    last = max(last, e)
    busy[nm(r)] += (e - s) / 1e3
    cnt[nm(r)] += 1
print(f"chol span {(int(rows[end]['Start_Timestamp']) - t0) / 1e3:.1f} us, gaps {gap:.1f} us")
for k, v in sorted(busy.items(), key=lambda x: -x[1]):
    print(f"  {v:8.1f} us {cnt[k]:4d}x avg {v / cnt[k]:6.2f}  {k}")
for r in rows[i0:i0 + 12]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    print(f"{s / 1e3:8.1f} {e / 1e3:8.1f} {(e - s) / 1e3:6.1f} {nm(r)}")
