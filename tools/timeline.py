"""Lay a protocol run's host chains against the GPU kernels they waited for.

Inputs (one run, same clock): the libmpcx_host timeline (MPCX_HOST_TRACE=<file>:
chain,kind,n,t0_ns,t1_ns -- rounds, rounds4_9 and every gpu.* call of a chain)
and the libmpcx kernel trace (MPCX_KTRACE=<file>, with the "kernel_stats" option
on: dev,kind,geom,ops,t0_ns,t1_ns).

    python tools/timeline.py host_trace.csv ktrace.csv [window_label] > summary.json

Reports, over the window spanned by the host trace's round intervals:
  - GPU busy share (union of kernel intervals) and the time-weighted number of
    kernels in flight, per kernel kind/geometry share;
  - per chain (one ordered signer pair of one wallet chunk): span, the share of
    it spent inside gpu.* calls (waiting on launches) and on the host;
  - per round: mean wall time, and within it the gpu-call / host split;
  - gpu.* calls: mean call time against the mean duration of the kernels that
    ran during it (queueing + coalescer wait + copies show as the difference).
"""
import collections
import csv
import json
import sys


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(iv):
    return sum(b - a for a, b in iv)


def clip(iv, lo, hi):
    return [(max(a, lo), min(b, hi)) for a, b in iv if b > lo and a < hi]


def main():
    host = list(csv.DictReader(open(sys.argv[1])))
    kern = list(csv.DictReader(open(sys.argv[2])))
    for r in host:
        r["t0"], r["t1"], r["chain"] = int(r["t0_ns"]) / 1e9, int(r["t1_ns"]) / 1e9, int(r["chain"])
    for r in kern:
        r["t0"], r["t1"] = int(r["t0_ns"]) / 1e9, int(r["t1_ns"]) / 1e9
    runs = [r for r in host if r["kind"] == "run"]
    if runs:  # the last traced run only (a line's warm-up run comes first)
        lo, hi = runs[-1]["t0"], runs[-1]["t1"]
        host = [r for r in host if r["kind"] != "run" and r["t0"] >= lo and r["t1"] <= hi]
    rounds = [r for r in host if not r["kind"].startswith("gpu.")]
    if not rounds:
        sys.exit("no round intervals in the host trace")
    if not runs:
        lo, hi = min(r["t0"] for r in rounds), max(r["t1"] for r in rounds)
    win = hi - lo
    kiv = clip([(r["t0"], r["t1"]) for r in kern], lo, hi)
    busy = length(union(kiv))
    # time-weighted kernels in flight while busy
    ev = sorted([(a, 1) for a, _ in kiv] + [(b, -1) for _, b in kiv])
    depth, last, hist = 0, lo, collections.Counter()
    for t, d in ev:
        if depth > 0:
            hist[depth] += t - last
        depth += d
        last = t
    inflight = sum(k * v for k, v in hist.items()) / max(busy, 1e-12)
    per_kind = collections.defaultdict(float)
    for r in kern:
        a, b = max(r["t0"], lo), min(r["t1"], hi)
        if b > a:
            per_kind[f'{r["kind"]}/g{r["geom"]}'] += b - a
    tot_k = sum(per_kind.values()) or 1e-12
    chains = collections.defaultdict(list)
    for r in host:
        chains[r["chain"]].append(r)
    per_chain = []
    round_stats = collections.defaultdict(lambda: {"n": 0, "wall": 0.0, "gpu": 0.0})
    for c, rs in sorted(chains.items()):
        rr = [r for r in rs if not r["kind"].startswith("gpu.")]
        gpu = [(r["t0"], r["t1"]) for r in rs if r["kind"].startswith("gpu.")]
        if not rr:
            continue
        a, b = min(r["t0"] for r in rr), max(r["t1"] for r in rr)
        g = length(union(clip(gpu, a, b)))
        per_chain.append({"chain": c, "span_s": round(b - a, 4), "gpu_wait_share": round(g / max(b - a, 1e-12), 3)})
        for r in rr:
            s = round_stats[r["kind"]]
            s["n"] += 1
            s["wall"] += r["t1"] - r["t0"]
            s["gpu"] += length(union(clip(gpu, r["t0"], r["t1"])))
    calls = collections.defaultdict(lambda: [0, 0.0])
    for r in host:
        if r["kind"].startswith("gpu."):
            calls[r["kind"]][0] += 1
            calls[r["kind"]][1] += r["t1"] - r["t0"]
    out = {
        "label": sys.argv[3] if len(sys.argv) > 3 else None,
        "window_s": round(win, 4),
        "gpu_busy_share": round(busy / win, 3),
        "kernels_in_flight_while_busy": round(inflight, 2),
        "in_flight_hist_s": {k: round(v, 4) for k, v in sorted(hist.items())},
        "kernel_time_share": {k: round(v / tot_k, 3) for k, v in sorted(per_kind.items(), key=lambda x: -x[1])},
        "rounds": {k: {"count": v["n"], "mean_wall_s": round(v["wall"] / v["n"], 4),
                       "gpu_wait_share": round(v["gpu"] / max(v["wall"], 1e-12), 3)} for k, v in round_stats.items()},
        "gpu_calls": {k: {"calls": n, "mean_ms": round(t / n * 1e3, 3)} for k, (n, t) in sorted(calls.items())},
        "chains": per_chain,
    }
    json.dump(out, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main()
