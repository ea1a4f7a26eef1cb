"""profiles/gram_pmc.json's "batched" entry from the counter CSVs of tools/pmc_gram.sh (dev tool):
python tools/gram_pmc_json.py <pmc_gram out dir> <source note>
Per width: fabric bytes (FETCH_SIZE x 2 on gfx950, KB x 1024, plus WRITE_SIZE) per Gram, MFMA busy,
clock (GRBM_GUI_ACTIVE / 8 / duration), L2 hit rate, ms per Gram of the PMC run."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

OUT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "gram_pmc.json")


def load(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)[0]
    val, dur = defaultdict(float), {}
    for r in csv.DictReader(open(f)):
        if "gram16b" not in r["Kernel_Name"]:
            continue
        val[r["Counter_Name"]] += float(r["Counter_Value"])
        dur[r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return val, dur


def main():
    root, note = sys.argv[1], sys.argv[2]
    per = {}
    for m, count in (("4096", 24), ("11008", 8)):
        mf, dm = load(os.path.join(root, f"g{m}_mfma"))
        fe, df = load(os.path.join(root, f"g{m}_fetch"))
        wr, _ = load(os.path.join(root, f"g{m}_write"))
        hi, _ = load(os.path.join(root, f"g{m}_hit"))
        grams = count * len(df)  # launches x items
        ns = sum(dm.values())
        cyc = mf["GRBM_GUI_ACTIVE"] / 8
        h, mi = hi.get("TCC_HIT_sum", 0), hi.get("TCC_MISS_sum", 0)
        per[m] = {"grams_per_launch_pmc_run": count,
                  "fabric_bytes_per_gram": (2 * fe["FETCH_SIZE"] * 1024 + wr["WRITE_SIZE"] * 1024) / grams,
                  "write_bytes_per_gram": wr["WRITE_SIZE"] * 1024 / grams,
                  "ms_per_gram_pmc_run": sum(df.values()) / 1e6 / grams,
                  "mfma_busy_frac": mf["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * 1024),
                  "clock_GHz": cyc / ns,
                  "l2_hit": h / (h + mi) if h + mi else None,
                  "algorithmic_bytes_per_gram": 2 * 262144 * int(m)}
    d = json.load(open(OUT))
    d["batched"] = {"kernel": "gram16b_kernel<false> (pt2q_gram_batched)", "source": note, "per_width": per}
    json.dump(d, open(OUT, "w"), indent=1)
    print(json.dumps(per, indent=1))


if __name__ == "__main__":
    main()
