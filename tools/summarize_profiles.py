"""Turn a profiling pass (tools/profile_round.sh -> gpurun_out/prof_<tag>/) into the tracked
summaries under profiles/:

  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats of `bench.py` (verbatim)
  profiles/<tag>_summary.md         top kernels + PMC-derived Gram figures
  profiles/gram_pmc.json            per-launch HBM-side bytes of the Gram (read by bench.py)

Counter handling follows /opt/skills/guides/MI355X_MICROARCH.md (HBM / rocprofv3 section):
FETCH_SIZE and WRITE_SIZE are in KB and were collected in separate passes; on gfx950 FETCH_SIZE
reports half the bytes of wide coalesced reads, so it is doubled.  Both count L2 <-> fabric
traffic, i.e. Infinity-Cache hits are included (an upper bound on DRAM bytes).
GRBM_GUI_ACTIVE is summed over the 8 XCDs; SQ_VALU_MFMA_BUSY_CYCLES is summed over SIMDs.

usage: python tools/summarize_profiles.py <tag> [bench_json]
"""
import csv
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GRAM = "gram16x_kernel"  # the 16-bit Gram (fp16/bf16 X); gram_streamk_kernel for f32 X
CUS, SIMDS, XCDS = 256, 4, 8


def pmc(src, counter):
    path = os.path.join(src, f"pmc_{counter}", "run_counter_collection.csv")
    vals = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if GRAM in r["Kernel_Name"]:
                key = r["Dispatch_Id"]
                vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    if not vals:
        raise SystemExit(f"no {GRAM} dispatch in {path}")
    return sum(vals.values()) / len(vals), len(vals)


def extra_counters(src):
    """Optional passes: L2 hit/miss and LDS bank conflicts of the Gram (per launch)."""
    out = {}
    for c in ("TCC_HIT_sum", "TCC_MISS_sum", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"):
        if os.path.exists(os.path.join(src, f"pmc_{c}", "run_counter_collection.csv")):
            out[c] = pmc(src, c)[0]
    if "TCC_HIT_sum" in out and "TCC_MISS_sum" in out:
        out["l2_hit_frac"] = out["TCC_HIT_sum"] / max(1.0, out["TCC_HIT_sum"] + out["TCC_MISS_sum"])
    return out


def gram_duration_ns(src, counter):
    path = os.path.join(src, f"pmc_{counter}", "run_kernel_trace.csv")
    ds = []
    with open(path) as f:
        for r in csv.DictReader(f):
            if GRAM in r["Kernel_Name"]:
                ds.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    return sum(ds) / len(ds)


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    out = os.path.join(ROOT, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(src, "trace", "run_kernel_stats.csv")
    shutil.copyfile(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))

    fetch_kb, n = pmc(src, "FETCH_SIZE")
    write_kb, _ = pmc(src, "WRITE_SIZE")
    busy, _ = pmc(src, "SQ_VALU_MFMA_BUSY_CYCLES")
    gui, _ = pmc(src, "GRBM_GUI_ACTIVE")
    dur_ns = gram_duration_ns(src, "GRBM_GUI_ACTIVE")
    cycles = gui / XCDS
    fetch_b = 2.0 * fetch_kb * 1024.0
    write_b = write_kb * 1024.0
    traffic = fetch_b + write_b
    mfma_util = busy / (cycles * CUS * SIMDS)
    rec = {
        "kernel": GRAM,
        "workload": "tools/bench_gram.py 262144 4096 fp16 (X 262144x4096 fp16 -> G 4096x4096 fp32)",
        "dispatches": n,
        "fetch_size_kb": fetch_kb,
        "write_size_kb": write_kb,
        "hbm_bytes_per_launch": traffic,
        "algorithmic_bytes_per_launch": 262144 * 4096 * 2 + 4096 * 4096 * 4,
        "avg_duration_ms_pmc_run": dur_ns / 1e6,
        "l2_fabric_GBps": traffic / dur_ns,
        "clock_GHz": cycles / dur_ns,
        "mfma_busy_frac": mfma_util,
        **extra_counters(src),
        "source": f"profiles/{tag}_summary.md: rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | "
                  "SQ_VALU_MFMA_BUSY_CYCLES | GRBM_GUI_ACTIVE, separate passes; "
                  "FETCH_SIZE x2 (gfx950), KB x1024; includes Infinity-Cache hits",
    }
    with open(os.path.join(out, "gram_pmc.json"), "w") as f:
        json.dump(rec, f, indent=1)

    rows = []
    with open(stats) as f:
        for r in csv.DictReader(f):
            rows.append(r)
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    lines = [f"# Profile {tag}", "",
             "Command: `rocprofv3 --kernel-trace --stats -- python3 bench.py --steps 3 --warmup 1 "
             "--no-cpu-baseline --no-n2048` (tools/profile_round.sh); full table in "
             f"`{tag}_kernel_stats.csv`.", "",
             "| kernel | calls | avg µs | total ms | % |", "|---|---|---|---|---|"]
    for r in rows[:15]:
        lines.append(f"| `{r['Name'][:90]}` | {r['Calls']} | {float(r['AverageNs']) / 1e3:.1f} | "
                     f"{float(r['TotalDurationNs']) / 1e6:.2f} | {float(r['Percentage']):.1f} |")
    lines += ["", "## Gram PMC (separate passes, `tools/bench_gram.py 262144 4096 fp16`)", ""]
    for k in ("fetch_size_kb", "write_size_kb", "hbm_bytes_per_launch", "algorithmic_bytes_per_launch",
              "avg_duration_ms_pmc_run", "l2_fabric_GBps", "clock_GHz", "mfma_busy_frac",
              "l2_hit_frac", "SQ_LDS_BANK_CONFLICT", "SQ_INSTS_LDS"):
        if k not in rec:
            continue
        v = rec[k]
        lines.append(f"- {k}: {v:.4g}" if isinstance(v, float) else f"- {k}: {v}")
    if len(sys.argv) > 2:
        with open(sys.argv[2]) as f:
            bench = f.read().strip()
        shutil.copyfile(sys.argv[2], os.path.join(out, f"{tag}_bench.json"))
        lines += ["", "## bench.py line (same round)", "", "```", bench, "```"]
    with open(os.path.join(out, f"{tag}_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    main()
