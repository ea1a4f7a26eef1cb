"""Per-kernel totals of a rocprofv3 kernel trace (dev tool):
python tools/kstats.py <run_kernel_trace.csv> [--after NAME_SUBSTR] [--top 30]

Prints total / count / average duration per kernel name and the span and busy time, optionally
only for the launches after the LAST launch whose name contains --after (e.g. to skip warmup)."""
import argparse
import csv
from collections import defaultdict


def short(name):
    return (name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--after", default=None)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    if a.after:
        idx = [i for i, r in enumerate(rows) if a.after in r["Kernel_Name"]]
        if idx:
            rows = rows[idx[-1] + 1:]
    tot, cnt = defaultdict(float), defaultdict(int)
    busy = 0.0
    for r in rows:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        tot[short(r["Kernel_Name"])] += d
        cnt[short(r["Kernel_Name"])] += 1
        busy += d
    span = (int(rows[-1]["End_Timestamp"]) - int(rows[0]["Start_Timestamp"])) / 1e3 if rows else 0
    print(f"launches {len(rows)}  span {span / 1e3:.2f} ms  kernel-busy {busy / 1e3:.2f} ms")
    for k, v in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
        print(f"{v / 1e3:10.3f} ms {cnt[k]:7d}x avg {v / cnt[k]:9.2f} us  {k}")


if __name__ == "__main__":
    main()
