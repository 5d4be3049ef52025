"""Per-kernel PMC summary of rocprofv3 --pmc passes (tools/gpu.sh pmc): every
counter averaged per dispatch of each kernel, plus the VALU issue rate.

    python tools/pmc_kernels.py OUT.json PASS_DIR [PASS_DIR ...] [--match SUBSTR ...]

GRBM_GUI_ACTIVE counts GPU-busy cycles summed over the 8 XCDs; a wave64 VALU
instruction holds a SIMD for 4 cycles, so SQ_INSTS_VALU / (GRBM_GUI_ACTIVE / 8
x 1024 SIMDs) is the wave-instructions per SIMD-cycle, 0.25 at the issue
ceiling. FETCH_SIZE / WRITE_SIZE are KB (uncorrected)."""
import collections
import csv
import glob
import json
import os
import sys


def short(name):
    return name.split("(")[0].replace("void ", "").replace("mpcx::", "").strip()


def main():
    args = sys.argv[1:]
    out, rest = args[0], args[1:]
    match = []
    if "--match" in rest:
        i = rest.index("--match")
        rest, match = rest[:i], rest[i + 1:]
    per = collections.defaultdict(lambda: collections.defaultdict(dict))  # kernel -> counter -> dispatch -> value
    for d in rest:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for row in csv.DictReader(open(f)):
                k = short(row.get("Kernel_Name", ""))
                if match and not any(m in k for m in match):
                    continue
                disp = (d, row.get("Dispatch_Id") or row.get("Correlation_Id"))
                c = row["Counter_Name"]
                per[k][c][disp] = per[k][c].get(disp, 0.0) + float(row["Counter_Value"])
    res = {}
    for k, cs in sorted(per.items()):
        r = {c: sum(v.values()) / len(v) for c, v in cs.items()}
        r["dispatches"] = max(len(v) for v in cs.values())
        g, vi = r.get("GRBM_GUI_ACTIVE"), r.get("SQ_INSTS_VALU")
        if g and vi:
            r["valu_wave_instr_per_simd_cycle"] = vi / (g / 8.0 * 1024.0)
            r["valu_issue_busy_frac"] = r["valu_wave_instr_per_simd_cycle"] / 0.25
        res[k] = r
    json.dump({"passes": rest, "kernels": res}, open(out, "w"), indent=1)
    for k, r in res.items():
        print(f"{k:45s} n={r['dispatches']:5d} VALU={r.get('SQ_INSTS_VALU', 0):.3e} "
              f"busy={r.get('valu_issue_busy_frac', float('nan')):.3f} fetchKB={r.get('FETCH_SIZE', float('nan')):.0f} "
              f"writeKB={r.get('WRITE_SIZE', float('nan')):.0f}")


if __name__ == "__main__":
    main()
