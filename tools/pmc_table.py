"""Per-dispatch PMC table for gpurun_out/pmcp (tools/pmc_probe16.sh): python tools/pmc_table.py [dir]"""
import csv, glob, os, sys
from collections import defaultdict
d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmcp"
vals = defaultdict(dict)
dur = {}
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        if "gram16" not in r["Kernel_Name"]:
            continue
        k = int(r["Dispatch_Id"])
        vals[k][r["Counter_Name"]] = vals[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
for f in sorted(glob.glob(os.path.join(d, "p*", "run_kernel_trace.csv"))):
    for r in csv.DictReader(open(f)):
        if "gram16" in r["Kernel_Name"]:
            dur.setdefault(os.path.dirname(f), []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
# dispatches are numbered per pass; group by order within the pass
bypass = defaultdict(list)
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    ids = sorted({int(r["Dispatch_Id"]) for r in csv.DictReader(open(f)) if "gram16" in r["Kernel_Name"]})
    rows = defaultdict(dict)
    for r in csv.DictReader(open(f)):
        if "gram16" in r["Kernel_Name"]:
            k = int(r["Dispatch_Id"])
            rows[k][r["Counter_Name"]] = rows[k].get(r["Counter_Name"], 0.0) + float(r["Counter_Value"])
    for pos, k in enumerate(ids):
        bypass[pos].append(rows[k])
for pos in sorted(bypass):
    merged = {}
    for x in bypass[pos]:
        merged.update(x)
    print(pos, {k: f"{v:.4g}" for k, v in sorted(merged.items())})
for k, v in dur.items():
    print(k, [f"{x/1e6:.2f}" for x in v])
