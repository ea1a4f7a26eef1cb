"""Concurrency view of a rocprofv3 kernel trace (dev tool):
python tools/overlap.py <run_kernel_trace.csv> [--top 25]

Sweeps the kernel intervals and prints: the span, the time covered by the Gram kernels, the
time covered by any kernel, the time spent with k kernels in flight, and each kernel's share of
the span when every instant is split evenly over the kernels running then ("wall share")."""
import argparse
import csv
from collections import defaultdict

from kstats import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--top", type=int, default=25)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ev = []
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        k = short(r["Kernel_Name"])
        ev.append((s, 1, k))
        ev.append((e, -1, k))
    ev.sort(key=lambda x: (x[0], x[1]))
    running = defaultdict(int)
    nrun = 0
    last = ev[0][0]
    share = defaultdict(float)
    conc = defaultdict(float)
    gram = 0.0
    for t, d, k in ev:
        dt = (t - last) / 1e3
        if dt > 0:
            conc[nrun] += dt
            if nrun:
                for name, c in running.items():
                    if c:
                        share[name] += dt * c / nrun
                if any(c and "gram16" in name for name, c in running.items()):
                    gram += dt
        last = t
        running[k] += d
        nrun += d
    span = (ev[-1][0] - ev[0][0]) / 1e3
    print(f"span {span / 1e3:.2f} ms; any kernel {(span - conc[0]) / 1e3:.2f} ms; "
          f"Gram running {gram / 1e3:.2f} ms")
    print("kernels in flight: " + ", ".join(f"{k}: {v / 1e3:.1f} ms" for k, v in sorted(conc.items())))
    for k, v in sorted(share.items(), key=lambda x: -x[1])[:a.top]:
        print(f"{v / 1e3:10.2f} ms wall share  {k}")


if __name__ == "__main__":
    main()
