"""Instruction census of a region of a hipcc -S listing (gfx950): counts by class.

    python tools/isa_census.py file.s START END [START END ...]
Classes: mad (v_mad_u64_u32 / v_mad_i64_i32), mfma, valu (other v_*), lds (ds_*), salu (s_*),
permlane / dpp are counted inside valu and also reported separately.
"""
import re
import sys
from collections import Counter


def census(lines):
    c = Counter()
    for ln in lines:
        t = ln.strip()
        if not t or t.startswith((";", ".")) or t.endswith(":"):
            continue
        op = t.split()[0]
        if op.startswith("v_mad_u64") or op.startswith("v_mad_i64"):
            c["mad"] += 1
        elif op.startswith("v_mfma"):
            c["mfma"] += 1
        elif op.startswith("v_"):
            c["valu"] += 1
            if "permlane" in op:
                c["permlane"] += 1
            if "dpp" in t or "row_" in t or "quad_perm" in t:
                c["dpp"] += 1
            c["v:" + op] += 1
        elif op.startswith("ds_"):
            c["lds"] += 1
            c["d:" + op] += 1
        elif op.startswith("s_"):
            c["salu"] += 1
            if op.startswith("s_nop"):
                c["s_nop"] += 1
            if op.startswith("s_waitcnt"):
                c["s_waitcnt"] += 1
        else:
            c["other:" + op] += 1
    return c


if __name__ == "__main__":
    src = open(sys.argv[1]).read().split("\n")
    args = list(map(int, sys.argv[2:]))
    for a, b in zip(args[::2], args[1::2]):
        c = census(src[a - 1:b])
        head = {k: c[k] for k in ("mad", "mfma", "valu", "permlane", "dpp", "lds", "salu", "s_nop", "s_waitcnt")}
        print(f"lines {a}-{b}: {head}")
        top = sorted(((v, k) for k, v in c.items() if k.startswith(("v:", "d:"))), reverse=True)[:25]
        print("   ", ", ".join(f"{k[2:]}={v}" for v, k in top))
