"""Per-phase kernel totals of the LAST grams-first step in a rocprofv3 kernel trace (dev tool):
python tools/phase_kstats.py <kernel_trace.csv> [--top 20]
Phases: gram (gram16* launches), inverse (after the last Gram up to the first block-loop kernel),
tails (the rest).  Prints the span, busy time and per-kernel totals of each phase."""
import os
import argparse
import csv
from collections import defaultdict

from kstats import short

LOOP = ("ssr_", "atq_", "ef_gemm")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=15)
    ap.add_argument("--json", default=None, help="also write {phase: {span_ms, busy_ms, kernels: {name: "
                                                 "[ms, launches]}}} here (bench.py's stage roofline reads it)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    def isg(r):
        return "gram16" in r["Kernel_Name"] or "gram_streamk" in r["Kernel_Name"]

    def neutral(r):  # torch elementwise ops and fills between the Grams (status OR, memsets)
        return "elementwise" in r["Kernel_Name"] or "fill" in r["Kernel_Name"].lower()
    # a step starts at a Gram whose previous non-neutral kernel is not a Gram
    steps, prev = [], None
    for i, r in enumerate(rows):
        if neutral(r):
            continue
        if isg(r) and (prev is None or not isg(prev)):
            steps.append(i)
        prev = r
    rows = rows[steps[-1]:]
    lastg = max(i for i, r in enumerate(rows) if isg(r))
    firstl = min(i for i, r in enumerate(rows) if i > lastg and any(k in r["Kernel_Name"] for k in LOOP))
    phases = {"gram": rows[:lastg + 1], "inverse": rows[lastg + 1:firstl], "tails": rows[firstl:]}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = {"source": os.path.relpath(os.path.abspath(a.csv), root) + " (kernel trace of tools/phase_times.py)"}
    for ph, rs in phases.items():
        if not rs:
            continue
        tot, cnt = defaultdict(float), defaultdict(int)
        busy = 0.0
        for r in rs:
            d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            tot[short(r["Kernel_Name"])] += d
            cnt[short(r["Kernel_Name"])] += 1
            busy += d
        span = (max(int(r["End_Timestamp"]) for r in rs) - int(rs[0]["Start_Timestamp"])) / 1e3
        print(f"== {ph}: launches {len(rs)}  span {span / 1e3:.2f} ms  kernel-busy {busy / 1e3:.2f} ms")
        out[ph] = {"span_ms": span / 1e3, "busy_ms": busy / 1e3, "launches": len(rs),
                   "kernels": {k: [v / 1e3, cnt[k]] for k, v in tot.items()}}
        for k, v in sorted(tot.items(), key=lambda x: -x[1])[:a.top]:
            print(f"{v / 1e3:10.3f} ms {cnt[k]:7d}x avg {v / cnt[k]:9.2f} us  {k}")
    if a.json:
        import json
        with open(a.json, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
