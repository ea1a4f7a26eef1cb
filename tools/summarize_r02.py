"""Turn the round-2 profiling pass (tools/profile_r02.sh -> gpurun_out/prof_<tag>/) into tracked
summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of one default-bench step
  profiles/<tag>_pmc.json           per-kernel PMC figures of each workload (per dispatch)
  profiles/<tag>_summary.md         the step's top kernels + the PMC table
  profiles/gram_pmc.json            per-launch fabric bytes of the Gram per width (bench.py)

Counter handling follows /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section): one
counter per run; FETCH_SIZE and WRITE_SIZE are in KB; on gfx950 FETCH_SIZE reports half the
bytes of wide coalesced reads, so it is doubled.  Both count L2 <-> fabric traffic (Infinity-Cache
hits included: an upper bound on DRAM bytes).  GRBM_GUI_ACTIVE is summed over the 8 XCDs;
SQ_VALU_MFMA_BUSY_CYCLES counts MFMA-busy cycles summed over the 1024 SIMDs.

usage: python tools/summarize_r02.py <tag>
"""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SIMDS, XCDS = 1024, 8
COUNTERS = ("FETCH_SIZE", "WRITE_SIZE", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE")
WORKLOADS = {
    "gram4096": "tools/bench_gram.py 262144 4096 fp16 (X 262144 x 4096 fp16 -> G 4096 x 4096)",
    "gram11008": "tools/bench_gram.py 262144 11008 fp16 (X 262144 x 11008 fp16 -> G 11008 x 11008)",
    "layer": "tools/run_layer.py 2 (fp16 4096 x 4096 layer, N = 262144, eager)",
    "chol": "tools/bench_chol.py 11008 (Cholesky inverse of an 11008 x 11008 damped Hessian)",
}


def short(name):
    return name.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]


def pass_values(d):
    """{kernel: [per-dispatch counter value]} and {kernel: [durations ns]} of one PMC pass."""
    vals, dur = defaultdict(dict), defaultdict(list)
    with open(os.path.join(d, "run_counter_collection.csv")) as f:
        for r in csv.DictReader(f):
            k = short(r["Kernel_Name"])
            did = r["Dispatch_Id"]
            vals[k][did] = vals[k].get(did, 0.0) + float(r["Counter_Value"])
    with open(os.path.join(d, "run_kernel_trace.csv")) as f:
        for r in csv.DictReader(f):
            dur[short(r["Kernel_Name"])].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return {k: list(v.values()) for k, v in vals.items()}, dur


def find(d):
    for root, _, files in os.walk(d):
        if "run_counter_collection.csv" in files:
            return root
    raise SystemExit(f"no counter csv under {d}")


def workload_table(src, wl):
    per = defaultdict(dict)
    for c in COUNTERS:
        vals, dur = pass_values(find(os.path.join(src, f"{wl}_{c}")))
        for k, v in vals.items():
            per[k][c] = sum(v) / len(v)
            per[k]["dispatches"] = len(v)
            if c == "GRBM_GUI_ACTIVE":
                per[k]["avg_ns"] = sum(dur[k]) / len(dur[k])
    out = {}
    for k, p in per.items():
        if not all(c in p for c in COUNTERS):
            continue
        ns = p["avg_ns"]
        cycles = p["GRBM_GUI_ACTIVE"] / XCDS
        byts = 2.0 * p["FETCH_SIZE"] * 1024.0 + p["WRITE_SIZE"] * 1024.0
        out[k] = {"dispatches": p["dispatches"], "avg_us": ns / 1e3, "fabric_bytes": byts,
                  "fabric_GBps": byts / ns, "clock_GHz": cycles / ns,
                  "mfma_busy_frac": p["SQ_VALU_MFMA_BUSY_CYCLES"] / max(1.0, cycles * SIMDS)}
    return out


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r02"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out = os.path.join(ROOT, "profiles")
    stats = os.path.join(find_stats(src), "run_kernel_stats.csv")
    shutil.copyfile(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    pmc = {wl: workload_table(src, wl) for wl in WORKLOADS}
    with open(os.path.join(out, f"{tag}_pmc.json"), "w") as f:
        json.dump({"workloads": WORKLOADS, "kernels": pmc}, f, indent=1)
    gram = {}
    for m in ("4096", "11008"):
        g = pmc[f"gram{m}"]
        k = [x for x in g if "gram16" in x][0]
        gram[m] = {"kernel": k, "fabric_bytes_per_launch": g[k]["fabric_bytes"], "avg_ms_pmc_run": g[k]["avg_us"] / 1e3,
                   "mfma_busy_frac": g[k]["mfma_busy_frac"], "clock_GHz": g[k]["clock_GHz"],
                   "algorithmic_bytes_per_launch": 262144 * int(m) * 2 + int(m) * int(m) * 4}
    with open(os.path.join(out, "gram_pmc.json"), "w") as f:
        json.dump({"kernel": "gram16x_kernel (m=4096) / gram16w_kernel (m=11008)", "per_width": gram,
                   "source": f"profiles/{tag}_summary.md: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | "
                             "SQ_VALU_MFMA_BUSY_CYCLES | GRBM_GUI_ACTIVE, separate passes; FETCH_SIZE "
                             "x2 (gfx950), KB x1024; includes Infinity-Cache hits"}, f, indent=1)
    rows = list(csv.DictReader(open(stats)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    L = [f"# Profile {tag}", "",
         "Kernel trace: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 1 --warmup 0 "
         "--no-cpu-baseline --no-extra` (one step = all 224 linears of the Llama-2-7B model; "
         f"tools/profile_r02.sh).  Kernel-busy total {tot / 1e9:.3f} s; full table in "
         f"`{tag}_kernel_stats.csv`.", "",
         "| kernel | calls | avg µs | total ms | % |", "|---|---|---|---|---|"]
    for r in rows[:20]:
        L.append(f"| `{short(r['Name'])}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                 f"{float(r['TotalDurationNs']) / 1e6:.1f} | {float(r['Percentage']):.1f} |")
    L += ["", "## PMC (one counter per run; per dispatch)", "",
          "fabric bytes = FETCH_SIZE x 2 + WRITE_SIZE (KB x 1024; L2 <-> fabric, Infinity-Cache hits "
          "included); MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs); "
          "clock = GRBM_GUI_ACTIVE / 8 / duration.  Durations are those of the PMC runs (serialised "
          "dispatches).  For short kernels (tens of µs) GRBM_GUI_ACTIVE also counts the dispatch's "
          "ramp-up and drain, so their GHz column reads above the real clock and their MFMA-busy "
          "fraction is a lower bound; the long kernels (Gram, gemmx) give the true figures.", ""]
    for wl, desc in WORKLOADS.items():
        L += [f"### {wl}: {desc}", "", "| kernel | dispatches | avg µs | fabric MB | GB/s | MFMA busy | GHz |",
              "|---|---|---|---|---|---|---|"]
        items = sorted(pmc[wl].items(), key=lambda kv: -kv[1]["avg_us"] * kv[1]["dispatches"])
        for k, v in items[:12]:
            L.append(f"| `{k}` | {v['dispatches']} | {v['avg_us']:.1f} | {v['fabric_bytes'] / 1e6:.1f} | "
                     f"{v['fabric_GBps']:.0f} | {v['mfma_busy_frac']:.3f} | {v['clock_GHz']:.2f} |")
        L.append("")
    with open(os.path.join(out, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(L) + "\n")
    print("\n".join(L))


def find_stats(src):
    for root, _, files in os.walk(os.path.join(src, "trace")):
        if "run_kernel_stats.csv" in files:
            return root
    raise SystemExit("no kernel stats")


if __name__ == "__main__":
    main()
