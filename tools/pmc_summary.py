"""Reduce rocprofv3 --pmc CSVs (gpurun_out/pmc/*) to per-launch numbers for
the k_modexp kernel: HBM bytes (FETCH_SIZE/WRITE_SIZE are KB), VALU
instructions, wave cycles, effective clock."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def load(pass_dir):
    vals = {}
    for f in glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                if "k_modexp" not in row.get("Kernel_Name", ""):
                    continue
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                vals.setdefault(row["Counter_Name"], {}).setdefault(d, 0.0)
                vals[row["Counter_Name"]][d] += float(row["Counter_Value"])
    return {k: sum(v.values()) / len(v) for k, v in vals.items() if v}, {k: len(v) for k, v in vals.items()}


def main(src=os.path.join(ROOT, "gpurun_out", "pmc"), label="k_modexp (bench config 2, 65536 x 4096-bit modexp, y=N)"):
    per = {}
    disp = {}
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        if os.path.isdir(d):
            v, n = load(d)
            per.update(v)
            disp.update(n)
    out = {"kernel": label,
           "per_launch_average": per, "dispatches_averaged": disp}
    if "FETCH_SIZE" in per and "WRITE_SIZE" in per:
        out["hbm_bytes_per_launch"] = (per["FETCH_SIZE"] + per["WRITE_SIZE"]) * 1024
        out["note"] = ("FETCH_SIZE/WRITE_SIZE are KB. The accesses are 4-B-per-lane buffer loads/stores (256 B per "
                       "wave-instruction): the guide's 2x FETCH_SIZE correction is calibrated for 16-B streaming "
                       "reads only, so it is not applied and the absolute is uncalibrated (MI355X_MICROARCH.md, HBM)")
    if "SQ_WAVE_CYCLES" in per and "GRBM_GUI_ACTIVE" in per:
        out["grbm_gui_active"] = per["GRBM_GUI_ACTIVE"]
    print(json.dumps(out, indent=1))
    return out


if __name__ == "__main__":
    # usage: pmc_summary.py [src_dir] [out_json] [label]
    a = sys.argv[1:]
    res = main(*( [a[0]] if a else []), *([a[2]] if len(a) > 2 else []))
    out = a[1] if len(a) > 1 else os.path.join(ROOT, "profiles", "r01", "pmc_summary.json")
    os.makedirs(os.path.dirname(out), exist_ok=True)
    json.dump(res, open(out, "w"), indent=1)
