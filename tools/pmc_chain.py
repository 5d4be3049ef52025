"""Reduce the rocprofv3 --pmc passes of the squaring-chain microbench
(tools/microbench/run_r6_occ.sh): per variant, the timed k_chain_mx dispatch's
counters (the largest SQ_WAVE_CYCLES, i.e. not the 2-squaring warm-up) and
per-wave-squaring figures.  usage: python tools/pmc_chain.py OUTDIR"""
import collections
import csv
import glob
import json
import os
import sys

out = {}
d = sys.argv[1]
for f in sorted(glob.glob(os.path.join(d, "pmc_*", "**", "*counter_collection.csv"), recursive=True)):
    var = os.path.relpath(f, d).split(os.sep)[0][4:-2]
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    names = {}
    for r in csv.DictReader(open(f)):
        if "chain_mx" not in r.get("Kernel_Name", ""):
            continue
        per[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    if not per:
        continue
    big = max(per.values(), key=lambda v: v.get("SQ_WAVE_CYCLES", 0) + v.get("GRBM_GUI_ACTIVE", 0))
    out.setdefault(var, {}).update({k: v for k, v in big.items()})
waves, sq = 4096, 64
for var, c in out.items():
    r = {}
    wc = c.get("SQ_WAVE_CYCLES")
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
        if wc and k in c:
            r[k + "_frac"] = round(c[k] / wc, 4)
    for k in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_INSTS_MFMA", "SQ_VALU_MFMA_BUSY_CYCLES"):
        if k in c:
            r[k + "_per_wave_sq"] = round(c[k] / waves / sq, 1)
    if "GRBM_GUI_ACTIVE" in c:
        r["clock_ghz_if_60ms"] = None
    c["derived"] = r
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(d, "pmc_summary.json"), "w"), indent=1)
