"""Symbolize and rank the host stack samples libmpcx_host writes under
MPCX_HOST_SAMPLE=<hz> MPCX_HOST_SAMPLE_OUT=<file> (hostprof.cpp sampler).

    python tools/host_samples.py gpurun_out/x/samples.3 [top] > summary.txt

Frames in this repo's .so files are symbolized with addr2line against the
local build (the box ran the same files); other modules keep module+offset
and are grouped per module. Prints self and inclusive sample shares per
function, innermost-frame first.
"""
import collections
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def local_path(mod):
    for marker in ("/mpcium_amd/",):
        if marker in mod:
            p = os.path.join(ROOT, "mpcium_amd", mod.split(marker, 1)[1])
            if os.path.exists(p):
                return p
    return None


def symbolize(frames):
    by_mod = collections.defaultdict(set)
    dyn = {}
    for f in frames:
        loc, _, sym = f.partition("@")
        mod, _, off = loc.rpartition("+")
        by_mod[mod].add(off)
        dyn[loc] = sym
    names = {}
    for mod, offs in by_mod.items():
        p = local_path(mod)
        offs = sorted(offs)
        if p is None:
            short = os.path.basename(mod) or "?"
            for o in offs:
                sym = dyn.get(f"{mod}+{o}")
                names[f"{mod}+{o}"] = f"[{short}{':' + sym if sym else ''}]"
            continue
        out = subprocess.run(["addr2line", "-f", "-C", "-e", p] + offs, capture_output=True, text=True).stdout
        lines = out.splitlines()
        for i, o in enumerate(offs):
            fn = lines[2 * i] if 2 * i < len(lines) else "??"
            names[f"{mod}+{o}"] = fn[:140] if fn != "??" else f"[{os.path.basename(mod)}+{o}]"
    return names


def main():
    path = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 40
    # --callers SUBSTR: the own-code frames above every sample whose stack holds SUBSTR
    callers = sys.argv[sys.argv.index("--callers") + 1] if "--callers" in sys.argv else None
    stacks = []
    for ln in open(path):
        c, _, st = ln.strip().partition(" ")
        if st:
            stacks.append((int(c), st.split(";")))
    names = symbolize({f for _, fr in stacks for f in fr})
    names = {f: names[f.partition("@")[0]] for _, fr in stacks for f in fr}
    total = sum(c for c, _ in stacks)
    self_c, own, incl = collections.Counter(), collections.Counter(), collections.Counter()
    if callers:
        chains = collections.Counter()
        for c, fr in stacks:
            syms = [names[f] for f in fr]
            hit = [i for i, s in enumerate(syms) if callers in s]
            if hit:
                up = [s.split("(")[0][-60:] for s in syms[hit[0]:] if not s.startswith("[")][:5]
                chains[" <- ".join(up)] += c
        n = sum(chains.values())
        print(f"{n} of {total} samples hold {callers!r}")
        for s, c in chains.most_common(top):
            print(f"{100.0 * c / total:6.2f}%  {s}")
        return
    for c, fr in stacks:
        syms = [names[f] for f in fr]
        self_c[syms[0]] += c
        # innermost frame in this repo's code, with the library frame it called
        for i, s in enumerate(syms):
            if not s.startswith("["):
                own[s + (f"  -> {syms[i - 1]}" if i else "")] += c
                break
        for s in set(syms):
            incl[s] += c
    print(f"{total} samples")
    print("-- self")
    for s, c in self_c.most_common(top):
        print(f"{100.0 * c / total:6.2f}%  {s}")
    print("-- innermost own frame (-> the library it was in)")
    for s, c in own.most_common(top):
        print(f"{100.0 * c / total:6.2f}%  {s}")
    print("-- inclusive")
    for s, c in incl.most_common(top):
        print(f"{100.0 * c / total:6.2f}%  {s}")


if __name__ == "__main__":
    main()
