"""Per-kernel summary of rocprofv3 --pmc runs with several counters per pass (dev tool):
python tools/pmc_multi.py <run dir> [<run dir> ...]
clock = GRBM_GUI_ACTIVE / 8 / duration; MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (cycles x 1024)
(256 CUs x 4 SIMDs); FETCH_SIZE x 2 (gfx950) and KB x 1024 (MI355X_MICROARCH.md); SQ_WAIT_* /
SQ_ACTIVE_INST_ANY as shares of SQ_WAVE_CYCLES."""
import csv
import glob
import os
import sys
from collections import defaultdict


def short(n):
    return n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:48]


def main():
    for d in sys.argv[1:]:
        f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
        val = defaultdict(lambda: defaultdict(float))
        dur = defaultdict(dict)
        for r in csv.DictReader(open(f)):
            k = short(r["Kernel_Name"])
            val[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        print(f"== {os.path.basename(d.rstrip('/'))}")
        rows = sorted(val, key=lambda k: -sum(dur[k].values()))
        for k in rows[:8]:
            ns = sum(dur[k].values())
            if ns < 1e5:
                continue
            c = val[k]
            out = [f"{k:48s} {len(dur[k]):5d}x {ns / 1e6:9.2f} ms"]
            cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8
            if cyc:
                out.append(f"clk {cyc / ns:.2f}GHz")
                if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    out.append(f"mfma {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
                if "SQ_BUSY_CYCLES" in c:
                    out.append(f"sqbusy {c['SQ_BUSY_CYCLES'] / (cyc * 8):.2f}")
            if "FETCH_SIZE" in c:
                b = 2 * c["FETCH_SIZE"] * 1024
                out.append(f"fetch {b / 1e9:.2f}GB {b / ns:.0f}GB/s")
            if "WRITE_SIZE" in c:
                b = c["WRITE_SIZE"] * 1024
                out.append(f"write {b / 1e9:.2f}GB {b / ns:.0f}GB/s")
            if "SQ_WAVE_CYCLES" in c and c["SQ_WAVE_CYCLES"]:
                w = c["SQ_WAVE_CYCLES"]
                for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_WAIT_INST_LDS"):
                    if n in c:
                        out.append(f"{n[3:].lower()} {c[n] / w:.2f}")
            if c.get("SQ_INSTS_VALU") and cyc:
                # a SIMD-32 issues one wave64 VALU instruction per 2 cycles: 1024 SIMDs x cycles / 2
                out.append(f"valu_insts {c['SQ_INSTS_VALU']:.3g} valu_issue_frac "
                           f"{c['SQ_INSTS_VALU'] / (cyc * 1024 / 2):.3f}")
                for n in ("SQ_INSTS_VMEM", "SQ_ACTIVE_INST_VALU"):
                    if n in c:
                        out.append(f"{n[3:].lower()} {c[n]:.3g}")
            if c.get("SQ_INSTS_LDS"):
                out.append(f"lds_insts {c['SQ_INSTS_LDS']:.3g}")
                if "SQ_LDS_BANK_CONFLICT" in c:
                    out.append(f"lds_conflict_cyc {c['SQ_LDS_BANK_CONFLICT']:.3g}")
                if c.get("SQ_LDS_IDX_ACTIVE"):
                    out.append(f"lds_conflict_share {c.get('SQ_LDS_BANK_CONFLICT', 0) / c['SQ_LDS_IDX_ACTIVE']:.3f}")
            print("  " + "  ".join(out))


if __name__ == "__main__":
    main()
