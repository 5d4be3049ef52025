"""Census every innermost loop of one kernel in a hipcc -S listing.

    python tools/isa_loops.py file.s KERNEL_SUBSTRING
A loop is a '.LBBx_y:' label marked 'Loop Header' up to the last branch back to it.
"""
import re
import sys

sys.path.insert(0, __import__("os").path.dirname(__file__))
from isa_census import census  # noqa: E402

src = open(sys.argv[1]).read().split("\n")
name = sys.argv[2]
start = next(i for i, l in enumerate(src) if l.startswith("_Z") and name in l and l.rstrip().endswith(":") or
             (l.startswith("_Z") and name in l.split(":")[0]))
end = next(i for i in range(start, len(src)) if src[i].strip().startswith(".Lfunc_end"))
body = src[start:end]
meta = [l for l in src if name in l and (".num_vgpr," in l or "private_seg_size" in l)]
print("\n".join(m.strip() for m in meta))
for i, l in enumerate(body):
    m = re.match(r"^(\.LBB\d+_\d+):.*Loop Header", l)
    if not m and "Loop Header" in l and i > 0:
        m = re.match(r"^(\.LBB\d+_\d+):", body[i - 1])
    if not m:
        continue
    lab = m.group(1)
    back = [j for j in range(i, len(body)) if re.search(r"s_cbranch_\w+\s+" + re.escape(lab) + r"$", body[j]) or
            re.search(r"s_branch\s+" + re.escape(lab) + r"$", body[j])]
    if not back:
        continue
    c = census(body[i:back[-1] + 1])
    print(lab, f"lines {start + i + 1}-{start + back[-1] + 1}",
          {k: c[k] for k in ("mad", "mfma", "valu", "dpp", "permlane", "lds", "salu", "s_nop", "s_waitcnt")})
