"""Condense an interleaved A/B directory (tools/gpu.sh ab/abswap/envab) into
one summary.json under profiles/: per-run headline values plus per-side means.

    python tools/ab_summary.py gpurun_out/r03/prime_ab profiles/r03/prime_ab/summary.json \
        "bash tools/gpu.sh abswap ..." ["A label" "B label" ...]   (abn: one label per build)
"""
import glob
import json
import os
import re
import sys

FIELDS = (
    ("config2_modexp_per_s", lambda d: round(d["value"])),
    ("config2_frac", lambda d: round(d["roofline"]["frac"], 4)),
    ("signing_2", lambda d: d["signing"]["value"]),
    ("signing_2_host_cpu_s", lambda d: d["signing"].get("host_cpu_s")),
    ("signing_3", lambda d: d["signing_3_signers"]["value"]),
    ("signing_3_host_cpu_s", lambda d: d["signing_3_signers"].get("host_cpu_s")),
    ("keygen", lambda d: d["keygen"]["value"]),
    ("safe_prime", lambda d: d["safe_prime"]["value"]),
    ("config2_kernel_ms", lambda d: round(d["roofline"]["kernel_ms"], 2)),
    ("per_operand_2048_kernel_ms", lambda d: round(d["config2_per_operand_exponents"][0]["kernel_ms"], 2)),
    ("paillier_batch", lambda d: d["paillier_batch"]["value"]),
    ("signing_2_kernel_frac", lambda d: round(d["signing"]["roofline"]["frac"], 4)),
    ("signing_3_kernel_frac", lambda d: round(d["signing_3_signers"]["roofline"]["frac"], 4)),
    ("keygen_kernel_frac", lambda d: round(d["keygen"]["roofline"]["frac"], 4)),
)


def row(path):
    d = json.load(open(path))
    out = {}
    for k, f in FIELDS:
        try:
            v = f(d)
        except (KeyError, TypeError):
            continue
        if v is not None:
            out[k] = round(v, 1) if isinstance(v, float) and abs(v) > 10 else v
    return out


def main():
    src, dst, cmd = sys.argv[1:4]
    labels = sys.argv[4:]
    runs, sides = [], {}
    for p in sorted(glob.glob(os.path.join(src, "ab_*.json"))):
        # ab_A_1 / ab_B_1 (ab, abswap, envab) or ab_L3_1 (abn: position in the build list)
        m = re.search(r"ab_([AB]|[LHE]\d+)_(\d+)\.json$", p)
        if not m:
            continue
        tag = m.group(1)
        k = "AB".index(tag) if tag in "AB" else int(tag[1:]) - 1
        side = labels[k] if k < len(labels) else tag
        r = {"run": f"{tag}_{m.group(2)}", "side": side}
        r.update(row(p))
        runs.append(r)
        sides.setdefault(side, []).append(r)
    runs.sort(key=lambda r: (int(r["run"].rsplit("_", 1)[1]), r["run"]))
    means = {}
    for s, rs in sides.items():
        keys = sorted({k for r in rs for k in r if k not in ("run", "side")})
        means[s] = {k: round(sum(r[k] for r in rs if k in r) / sum(1 for r in rs if k in r), 4) for k in keys}
    os.makedirs(os.path.dirname(dst), exist_ok=True)
    json.dump({"command": cmd, "runs": runs, "means": means}, open(dst, "w"), indent=1)
    print(json.dumps(means, indent=1))


if __name__ == "__main__":
    main()
