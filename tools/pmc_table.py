"""Per-kernel PMC table of a tools/pmc_gram.sh run (dev tool): python tools/pmc_table.py <dir>

One counter per run (<dir>/<CTR>/); FETCH_SIZE x 2 (gfx950) and KB x 1024 as in
tools/summarize_r02.py; L2 hit = TCC_HIT / (TCC_HIT + TCC_MISS); LDS conflict share =
SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from summarize_r02 import find, pass_values  # noqa: E402


def main():
    d = sys.argv[1]
    per = {}
    for ctr in sorted(os.listdir(d)):
        p = os.path.join(d, ctr)
        if not os.path.isdir(p):
            continue
        vals, dur = pass_values(find(p))
        for k, v in vals.items():
            e = per.setdefault(k, {})
            e[ctr] = sum(v) / len(v)
            e["ns"] = sum(dur[k]) / len(dur[k])
            e["n"] = len(v)
    for k, e in per.items():
        if "gram" not in k:
            continue
        ns = e["ns"]
        cyc = e.get("GRBM_GUI_ACTIVE", 0) / 8
        out = [f"{k}: {e['n']} dispatches, {ns / 1e6:.2f} ms"]
        if "FETCH_SIZE" in e:
            fb = 2 * e["FETCH_SIZE"] * 1024
            out.append(f"fetch {fb / 1e9:.1f} GB ({fb / ns:.0f} GB/s)")
        if "WRITE_SIZE" in e:
            out.append(f"write {e['WRITE_SIZE'] * 1024 / 1e9:.2f} GB")
        if cyc:
            out.append(f"clock {cyc / ns:.2f} GHz")
            if "SQ_VALU_MFMA_BUSY_CYCLES" in e:
                out.append(f"MFMA busy {e['SQ_VALU_MFMA_BUSY_CYCLES'] / (cyc * 1024):.3f}")
        if "TCC_HIT_sum" in e and "TCC_MISS_sum" in e:
            h, mi = e["TCC_HIT_sum"], e["TCC_MISS_sum"]
            out.append(f"L2 hit {h / max(1, h + mi):.3f} ({(h + mi) * 128 / 1e9:.0f} GB of 128-B requests)")
        if "SQ_LDS_BANK_CONFLICT" in e and "SQ_LDS_IDX_ACTIVE" in e:
            out.append(f"LDS conflict {e['SQ_LDS_BANK_CONFLICT'] / max(1, e['SQ_LDS_IDX_ACTIVE']):.3f}")
        print("; ".join(out))


if __name__ == "__main__":
    main()
