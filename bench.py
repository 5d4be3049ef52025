#!/usr/bin/env python3
"""bench.py -- BASELINE.json config 2 on MI355X.

Workload ("step" = one pass of the hot path over one batch): 65,536
modular exponentiations x^N mod N^2 (4096-bit modulus, shared 2048-bit
exponent y = N -- the r^N / s^N / beta^N shape of Paillier Encrypt and the
MtA proofs), bases uniform-ish below N^2 from a seeded generator, the node
key N from tests/golden/paillier_key_2048.json. Inputs are resident in HBM
before the timed region; one step = one libmpcx kernel launch over the batch.

Multi-GPU (torchrun, one process per GPU): every rank runs its own 65,536
operands (independent sessions shard with no exchange step -> weak scaling,
no collective on the data path); `value` = all ranks' modexps / max time.

Prints ONE JSON line on rank 0 (contract in the task statement), with
`roofline` (INT32 VALU bound, algorithmic work of Go's 4-bit-window
Montgomery ladder) and `cpu_baseline` (the C restatement of Go
expNNMontgomery timed on this host's cores, rank 0, N=1 only).
"""
from __future__ import annotations

import argparse
import collections
import json
import math
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "4096-bit modexp/s per GPU & node; 2-of-3 ECDSA sigs/s over 10k wallets"
PEAK_INT32_NOMINAL = 256 * 64 * 2.4e9  # 39.3 T 32x32->64 MAC/s: v_mad_u64_u32 is half rate on gfx950
PEAK_MAD_MEASURED = 33.8e12            # tools/microbench/valu_rates.hip, 8 waves/SIMD (profiles/r01_valu_rates.txt)




PMC_TRAFFIC = os.path.join(ROOT, "profiles", "r05", "pmc", "config2_traffic.json")        # k_modexp<4, 37, 16, 2>
PMC_TRAFFIC_MX = os.path.join(ROOT, "profiles", "r06", "pmc_mx", "config2_traffic.json")  # k_modexp_mx


def pmc_traffic(count: int, modbits: int, mod, mx: bool = False) -> dict:
    """roofline.traffic: fabric bytes per launch of the bench kernel from the
    committed rocprofv3 FETCH_SIZE and WRITE_SIZE passes (separate --pmc runs of
    the bench command over the current kernel, tools/gpu.sh pmc). rocprofv3 cannot run
    inside the timed process. Only reported for the workload those passes
    measured (65,536 operands, 4096-bit modulus, 4x37 quad geometry); null
    otherwise. The algorithmic I/O is 1 KB per operand (base in, result out).
    Most FETCH bytes are window-table re-reads that miss the per-XCD L2
    (DESIGN.md 5.4); the memory-side counters include Infinity-Cache hits, so
    this is an upper bound on HBM bytes."""
    out = {"traffic": None, "traffic_unit": "bytes/launch", "algorithmic_io_bytes": count * 2 * modbits // 8}
    path = PMC_TRAFFIC_MX if mx else PMC_TRAFFIC
    if count != 65536 or modbits != 4096 or (mod.P, mod.K) != (4, 37) or not os.path.exists(path):
        return out
    with open(path) as f:
        s = json.load(f)
    out["traffic"] = s["hbm_bytes_per_launch"]
    out["traffic_source"] = (os.path.relpath(path, ROOT) + f" ({s.get('kernel')}; 2 x FETCH_SIZE + WRITE_SIZE: the "
                             "counters' calibration on this access width, tools/microbench/fetch_calib.hip)")
    return out

# GPU clock / power / temperature sampler: a separate process (started before
# this one touches the GPU) that reads the amdsmi GPU metrics of one device every
# `interval` seconds and appends one JSON line per sample (wall time "t") until
# its stdin closes. bench.py keeps the samples inside its timed region.
SMI_SAMPLER = r"""
import json, select, sys, time
bdf, interval, path = sys.argv[1], float(sys.argv[2]), sys.argv[3]
import amdsmi
amdsmi.amdsmi_init()
hs = amdsmi.amdsmi_get_processor_handles()
h = hs[0] if hs else None
for x in hs:
    try:
        if bdf and amdsmi.amdsmi_get_gpu_device_bdf(x).lower().endswith(bdf.lower()):
            h = x
            break
    except Exception:
        pass
KEEP = ("clk", "power", "temperature", "throttle", "activity", "energy")
with open(path, "w") as f:
    while h is not None:
        rec = {"t": time.time()}
        try:
            m = amdsmi.amdsmi_get_gpu_metrics_info(h)
            for k, v in m.items():
                if not any(s in k for s in KEEP):
                    continue
                if isinstance(v, (int, float)):
                    rec[k] = v
                elif isinstance(v, list):
                    nums = [y for y in v if isinstance(y, (int, float)) and y not in (65535, 0xFFFFFFFF)]
                    if nums:
                        rec[k] = nums
        except Exception as e:
            rec["error"] = repr(e)[:200]
        f.write(json.dumps(rec) + "\n")
        f.flush()
        r, _, _ = select.select([sys.stdin], [], [], interval)
        if r and not sys.stdin.read(1):
            break
amdsmi.amdsmi_shut_down()
"""


class SmiSampler:
    """Runs SMI_SAMPLER beside the benchmark (a child process started before
    the GPU is initialised in this process) and summarises the samples that
    fall inside a wall-clock window."""

    def __init__(self, gpu: int, interval: float = 0.1):
        import subprocess
        import tempfile
        self.path = os.path.join(tempfile.gettempdir(), f"mpcx_smi_{os.getpid()}.jsonl")
        bdf = ""
        try:  # match the HIP ordinal to its amdsmi handle by PCI bus id (no GPU init needed)
            ids = sorted(os.listdir("/sys/bus/pci/drivers/amdgpu"))
            ids = [i for i in ids if i.count(":") == 2]
            vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("ROCR_VISIBLE_DEVICES")
            if vis:
                ids = [ids[int(v)] for v in vis.split(",") if v.strip().isdigit() and int(v) < len(ids)]
            bdf = ids[gpu] if gpu < len(ids) else ""
        except OSError:
            pass
        self.bdf = bdf
        try:
            self.proc = subprocess.Popen([sys.executable, "-c", SMI_SAMPLER, bdf, str(interval), self.path],
                                         stdin=subprocess.PIPE, stdout=subprocess.DEVNULL,
                                         stderr=subprocess.DEVNULL)
        except OSError:
            self.proc = None

    def stop(self):
        if self.proc is None:
            return
        try:
            self.proc.stdin.close()
            self.proc.wait(timeout=10)
        except Exception:
            self.proc.kill()

    def window(self, t0: float, t1: float) -> dict | None:
        """Mean / min / max of every sampled metric with t in [t0, t1], plus
        the first and last sample of the window (drift over the run)."""
        try:
            recs = [json.loads(x) for x in open(self.path) if x.strip()]
        except (OSError, ValueError):
            return None
        win = [r for r in recs if t0 <= r["t"] <= t1]
        if not win:
            return {"samples": 0, "samples_total": len(recs), "bdf": self.bdf,
                    "error": (recs[0].get("error") if recs else "no samples")}
        out = {"samples": len(win), "bdf": self.bdf, "interval_s": (t1 - t0) / max(1, len(win))}
        keys = sorted({k for r in win for k in r if k not in ("t", "error")})
        for k in keys:
            vals = []
            for r in win:
                v = r.get(k)
                if isinstance(v, list):
                    v = sum(v) / len(v)
                if isinstance(v, (int, float)):
                    vals.append(float(v))
            if vals:
                out[k] = {"mean": sum(vals) / len(vals), "min": min(vals), "max": max(vals),
                          "first": vals[0], "last": vals[-1]}
        return out


def gpu_index() -> int:
    """This rank's GPU: LOCAL_RANK, wrapped onto the visible devices so a
    multi-rank rehearsal also runs on a one-GPU box (the driver's N-GPU runs
    have one device per local rank, so this is the identity there).
    torch.cuda.device_count() does not initialise the GPU on this image."""
    import torch
    return int(os.environ.get("LOCAL_RANK", "0")) % max(1, torch.cuda.device_count())

PEAK_I8_MFMA = 256 * 4 * 1024 * 2.4e9  # 2.5 P i8 MAC/s dense: 16x16x64 i8 = 16 cycles per SIMD


def sliding_window_counts(e: int, width: int = 6):
    """(squarings, table products, window products) of a left-to-right sliding
    window over e with windows of up to `width` bits (k_expsched's schedule shape)."""
    bits = bin(e)[2:]
    i, sq, wins, top = 0, 0, 0, 0
    first = True
    while i < len(bits):
        if bits[i] == "0":
            sq += 0 if first else 1
            i += 1
            continue
        j = min(len(bits), i + width)
        while bits[j - 1] == "0":
            j -= 1
        v = int(bits[i:j], 2)
        top = max(top, v)
        if first:
            first = False
        else:
            sq += j - i
            wins += 1
        i = j
    return sq, (top - 1) // 2 + 1, wins


def mx_floor(count: int, e: int, kernel_ms: float) -> dict:
    """Resource floor of the work k_modexp_mx EXECUTES for count x x^e mod a 4096-bit
    modulus: the product loop's v_mad_u64_u32 lane-MADs (148 iterations x 19 per lane
    for a squaring, x 37 for a product, 4 lanes per operand) at the INT32 MAD peak,
    and the reduction's i8 MACs (417 16x16x64 MFMAs per 16 operands per product) at
    the dense i8 matrix peak. Everything else the kernel issues (carries, radix
    conversions, normalisation, LDS traffic) is overhead over this floor."""
    sq, tab, wins = sliding_window_counts(e)
    sq += 1                      # x^2 R for the odd-power chain
    prods = 1 + (tab - 1) + wins  # x R, the odd powers, the window multiplies (the exit runs on the CIOS loop)
    valu = count * (sq * 148 * 19 * 4 + prods * 148 * 37 * 4)
    i8 = count * (sq + prods) * 417 * 16384 / 16
    t_valu, t_mfma = valu / PEAK_INT32_NOMINAL, i8 / PEAK_I8_MFMA
    floor = max(t_valu, t_mfma)
    return {"kernel": "k_modexp_mx (Montgomery reduction on v_mfma_i32_16x16x64_i8, mpcx_mx.hpp)",
            "squarings": sq, "products": prods, "valu_lane_mads": valu, "mfma_i8_macs": i8,
            "floor_ms_valu": t_valu * 1e3, "floor_ms_mfma": t_mfma * 1e3,
            "frac_of_floor": floor / (kernel_ms * 1e-3),
            "note": "frac_of_floor = the executed work's resource floor (its MADs at the INT32 MAD peak, "
                    "its i8 MACs at the dense i8 MFMA peak, whichever is longer) over the launch time; the "
                    "headline frac keeps the rounds' algorithmic definition (Go-equivalent 32-bit MACs at the "
                    "INT32 MAD peak), which the matrix cores let exceed what a VALU-only kernel could reach"}


def two_pipe_roofline(r: dict) -> None:
    """k_modexp_mx runs on two pipes (VALU product loop, i8 matrix-core reduction),
    so the INT32-VALU ratio of the Go-equivalent work can pass 1 and is no
    utilisation. In place: `frac` becomes the executed work's
    floor over the launch (its VALU lane-MADs at the INT32 MAD peak or its i8 MACs
    at the dense i8 peak, whichever binds; <= 1), `achieved`/`peak` the binding
    pipe's executed rate and peak, `bound` "valu+mfma_i8"; the rounds' algorithmic
    ratio moves to the go_equiv_* keys, the other pipe's rate beside it."""
    ef = r["executed_floor"]
    t = r["kernel_ms"] * 1e-3
    valu_rate, i8_rate = ef["valu_lane_mads"] / t, ef["mfma_i8_macs"] / t
    valu_binds = ef["floor_ms_valu"] >= ef["floor_ms_mfma"]
    r["go_equiv_achieved"], r["go_equiv_peak"], r["go_equiv_frac"] = r["achieved"], r["peak"], r["frac"]
    r["go_equiv_note"] = ("Go-equivalent 32-bit MACs (SURVEY 8(d): (E + E/4) 2 L^2 per modexp) per second against "
                          "the INT32 MAD peak: the rounds' throughput ratio, not a utilisation once the matrix "
                          "cores take the reduction")
    if "frac_at_measured_clock" in r:
        r["go_equiv_frac_at_clock"] = r.pop("frac_at_measured_clock")
    r["bound"] = "valu+mfma_i8"
    r["binding_pipe"] = "valu" if valu_binds else "mfma_i8"
    r["achieved_valu"], r["peak_valu"] = valu_rate / 1e12, PEAK_INT32_NOMINAL / 1e12
    r["achieved_i8"], r["peak_i8"] = i8_rate / 1e12, PEAK_I8_MFMA / 1e12
    r["frac_valu"], r["frac_i8"] = valu_rate / PEAK_INT32_NOMINAL, i8_rate / PEAK_I8_MFMA
    r["achieved"], r["peak"] = (r["achieved_valu"], r["peak_valu"]) if valu_binds else (r["achieved_i8"], r["peak_i8"])
    r["frac"] = ef["frac_of_floor"]
    r["unit"] = "TOP/s"
    clk = r.get("gfxclk_mhz_measured")
    if clk:
        r["frac_at_clock"] = r["frac"] * 2400.0 / clk


def alg_macs(mod_bits: int, exp_bits: int) -> float:
    """W = (E + ceil(E/4)) * 2 L^2 32-bit MACs, L = 32-bit limbs."""
    L = math.ceil(mod_bits / 32)
    return (exp_bits + math.ceil(exp_bits / 4)) * 2 * L * L


def load_key():
    with open(os.path.join(ROOT, "tests", "golden", "paillier_key_2048.json")) as f:
        k = json.load(f)
    return int(k["N"], 16)


def synth_bases(N2: int, count: int, seed: int, words: int) -> np.ndarray:
    """count x words little-endian uint32, each value < N^2 (top word clamped)."""
    rng = np.random.default_rng(seed)
    x = rng.integers(0, 1 << 32, size=(count, words), dtype=np.uint64).astype(np.uint32)
    top = (N2 >> (32 * (words - 1))) & 0xFFFFFFFF
    x[:, words - 1] = x[:, words - 1] % max(top, 1)
    return x


def host_info() -> dict:
    """The host the CPU baseline ran on: nproc, this process's CPU affinity,
    the cgroup CPU quota (a GPU box gives a job a share of the machine:
    os.cpu_count() shows every CPU, the quota what may run at once) and the CPU
    model. usable_threads = min(affinity, quota): the CPU legs run there."""
    info = {"nproc": os.cpu_count(), "affinity": len(os.sched_getaffinity(0)), "cgroup_quota_cpus": None,
            "cpu_model": None}
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            a, b = f.read().split()[:2]
        if a != "max":
            info["cgroup_quota_cpus"] = int(a) / int(b)
    except (OSError, ValueError):
        pass
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    info["cpu_model"] = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    usable = info["affinity"]
    if info["cgroup_quota_cpus"]:
        usable = min(usable, max(1, int(info["cgroup_quota_cpus"])))
    info["usable_threads"] = usable
    return info


_C_SECONDS = collections.defaultdict(float)  # thread ident -> seconds inside the C restatement's calls


def _c_call(fn, *a):
    """Call the C restatement, adding its duration to this thread's C time
    (python_share of the CPU legs = the rest of the threads' time)."""
    t0 = time.perf_counter()
    r = fn(*a)
    _C_SECONDS[threading.get_ident()] += time.perf_counter() - t0
    return r


def _time_threads(make_work, seconds: float, threads: int):
    """Run make_work(t)() repeatedly on `threads` Python threads (the work is
    a ctypes call that releases the GIL) for `seconds`; -> (ops, elapsed)."""
    _C_SECONDS.clear()
    done = [0] * threads
    stop = time.perf_counter() + seconds

    def run(t):
        w = make_work(t)
        while time.perf_counter() < stop:
            w()
            done[t] += 1

    t0 = time.perf_counter()
    ths = [threading.Thread(target=run, args=(i,)) for i in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    return sum(done), time.perf_counter() - t0


_LAST_PYTHON_SHARE = [None]


def _one_and_all(make_work, seconds: float, info: dict):
    """1-thread and all-usable-thread rates of the same work (seconds split 1:2).
    _LAST_PYTHON_SHARE[0]: the all-thread run's share of thread time outside
    the C calls (Python orchestration and conversions, GIL waits)."""
    n1, e1 = _time_threads(make_work, seconds / 3, 1)
    thr = info["usable_threads"]
    nn, en = _time_threads(make_work, 2 * seconds / 3, thr) if thr > 1 else (n1, e1)
    _LAST_PYTHON_SHARE[0] = max(0.0, 1.0 - sum(_C_SECONDS.values()) / (thr * en)) if _C_SECONDS else None
    return n1 / e1, nn / en, thr, (n1, e1, nn, en)


def cpu_baseline(N: int, seconds: float, info: dict):
    """Config 2 on this host's cores: x^N mod N^2 by the C restatement of Go
    expNNMontgomery with Go's amd64 64-bit Words (oracle/libgomodexp64.so,
    `value`, one thread and all usable threads), GMP mpz_powm (a faster proxy
    for math/big) and the 32-bit-word restatement alongside."""
    import ctypes
    from oracle import crosscheck as cc  # test infrastructure: cpu_baseline leg only
    lib64, lib32 = cc.load_c_oracle(64), cc.load_c_oracle(32)
    if lib64 is None:
        return None
    N2 = N * N
    nw = (N2.bit_length() + 31) // 32
    ew = (N.bit_length() + 31) // 32
    mw = cc._words(N2, nw)
    yw = cc._words(N, ew)

    def c_work(lib):
        def make(t):
            rng = np.random.default_rng(7 + t)
            out = (ctypes.c_uint32 * nw)()
            xs = rng.integers(0, 1 << 32, size=nw, dtype=np.uint64).astype(np.uint32)
            xs[-1] = xs[-1] % max((N2 >> (32 * (nw - 1))), 1)
            xw = (ctypes.c_uint32 * nw)(*[int(v) for v in xs])
            return lambda: _c_call(lib.gomodexp_montgomery, out, xw, nw, yw, ew, mw, nw)
        return make

    r1, rn, thr, raw = _one_and_all(c_work(lib64), seconds * 0.5, info)
    out = {"value": rn, "unit": "modexp/s", "cores": thr, "kind": "port", "one_core": r1,
           "python_share": _LAST_PYTHON_SHARE[0],
           "all_cores_extrapolated": r1 * info["nproc"],
           "sample": f"{raw[2]} x (x^N mod N^2, 4096-bit modulus, 2048-bit exponent) in {raw[3]:.1f} s on {thr} "
                     f"threads (+ {raw[0]} on 1 thread in {raw[1]:.1f} s); C restatement of Go expNNMontgomery with "
                     f"Go's amd64 64-bit Words and 4-bit window (oracle/gomodexp.c -DGOMODEXP_W64); Go/tss-lib absent",
           "note": "value = all usable threads (min(affinity, cgroup quota)); all_cores_extrapolated = one_core x "
                   "nproc, the node's host capacity if every CPU ran this work at the one-thread rate",
           **info}
    g = cc.GmpPowm(1, N, N2)
    if g.ok:
        g.close()

        def gmp_make(t):
            import random
            rng = random.Random(31 + t)
            gp = cc.GmpPowm(rng.randrange(N2), N, N2)
            return gp.run
        g1, gn, gthr, graw = _one_and_all(gmp_make, seconds * 0.3, info)
        out["gmp_mpz_powm"] = {"one_core": g1, "value": gn, "cores": gthr, "version": cc.gmp_version(),
                               "all_cores_extrapolated": g1 * info["nproc"],
                               "sample": f"{graw[2]} mpz_powm in {graw[3]:.1f} s on {gthr} threads"}
    else:
        out["gmp_mpz_powm"] = None
    if lib32 is not None:
        n32, e32 = _time_threads(c_work(lib32), seconds * 0.2, 1)
        out["port_32bit_words_one_core"] = n32 / e32
    return out


def _c_exp_words(lib, nw):
    """x^y mod m through the C restatement of Go's expNNMontgomery (words in/out)."""
    import ctypes
    from oracle import crosscheck as cc

    def f(x, y, m):
        out = (ctypes.c_uint32 * nw)()
        ew = max(1, (y.bit_length() + 31) // 32)
        xw, yw, mw = cc._words(x, nw), cc._words(y, ew), cc._words(m, nw)
        _c_call(lib.gomodexp_montgomery, out, xw, nw, yw, ew, mw, nw)
        return int.from_bytes(bytes(out), "little")
    return f


def cpu_baseline_paillier(N: int, seconds: float, info: dict):
    """Config 1 on host cores: tss-lib Encrypt (Gamma^m r^N mod N^2) +
    HomoMult (c^b) with Go's expNNMontgomery restated in C (64-bit Words).
    `value`: tss-lib's own work (Gamma^m as a full Exp, as up:crypto/paillier
    does); `same_work_as_gpu`: with the GPU's bit-exact 1 + mN shortcut."""
    from oracle import crosscheck as cc
    lib = cc.load_c_oracle(64)
    if lib is None:
        return None
    N2 = N * N
    nw = (N2.bit_length() + 31) // 32
    exp = _c_exp_words(lib, nw)
    Q = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141

    def make(shortcut):
        def mk(t):
            import random
            rng = random.Random(11 + t)

            def one():
                m, r, b = rng.randrange(N), rng.randrange(1, N), rng.randrange(Q)
                gm = (1 + m * N) % N2 if shortcut else exp(N + 1, m, N2)
                c = gm * exp(r, N, N2) % N2
                exp(c, b, N2)
            return one
        return mk

    r1, rn, thr, raw = _one_and_all(make(False), seconds * 0.6, info)
    py_share = _LAST_PYTHON_SHARE[0]
    s1, sn, _, sraw = _one_and_all(make(True), seconds * 0.4, info)
    return {"value": rn, "unit": "Encrypt+HomoMult ops/s", "cores": thr, "kind": "port", "one_core": r1,
            "python_share": py_share,
            "all_cores_extrapolated": r1 * info["nproc"],
            "same_work_as_gpu": {"value": sn, "one_core": s1, "cores": thr,
                                 "all_cores_extrapolated": s1 * info["nproc"]},
            "sample": f"{raw[2]} x (Encrypt: Gamma^m and r^N mod N^2 as Exps; HomoMult: c^b, b < q) in {raw[3]:.1f} s "
                      f"on {thr} threads; same_work_as_gpu: Gamma^m = 1 + mN; oracle/gomodexp.c (64-bit Words)",
            **info}


def paillier_line(N: int, batch: int, reps: int, cpu: bool, info: dict, world: int = 1, rank: int = 0,
                  inflight: int = 16):
    """Config 1 (BASELINE.json): tss-lib paillier Encrypt + HomoMult over a
    batch of `batch` ops, 2048-bit N, through the host mirror of
    crypto/paillier (libmpcx_host.so -> libmpcx.so; host buffers, so the rate
    includes PCIe; operands cross as word arrays, converted from Python ints
    outside the timed loops). world > 1: every rank
    runs its own batches (weak scaling); value = all ranks' ops / max time."""
    import random
    from mpcium_amd import host as mhost
    from oracle import gomath as gm
    mhost.init(gpu_index())
    pk = mhost.PublicKey(N)
    rng = random.Random(0x6D706331 + 7919 * rank)
    Q = 0xFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFFEBAAEDCE6AF48A03BBFD25E8CD0364141
    ms = [rng.randrange(N) for _ in range(batch)]
    rs = [rng.randrange(1, N) for _ in range(batch)]
    bs = [rng.randrange(Q) for _ in range(batch)]
    cs, err = pk.encrypt(ms, rs)
    out, err2 = pk.homo_mult(bs, cs)
    if any(err) or any(err2):
        raise SystemExit("paillier line: error codes")
    for i in range(0, batch, max(1, batch // 8)):  # untimed spot check vs the oracle formulas
        if cs[i] != gm.paillier_encrypt(N, ms[i], rs[i]) or out[i] != gm.paillier_homo_mult(N, bs[i], cs[i]):
            raise SystemExit(f"paillier line: mismatch at {i}")
    if world > 1:
        import torch.distributed as dist
        from mpcium_amd.shard import max_over_ranks
        dist.barrier()
    # value: BASELINE.json configs[0] as stated -- ONE batch of 1,024 Encrypt +
    # HomoMult ops at a time, repeated `reps` times. The operands cross as word
    # arrays (host buffers, PCIe included), converted from Python ints once
    # before the timed region: the Python-int <-> words conversions (~9 ms per
    # batch in CPython) are the harness's, not the engine's.
    from mpcium_amd.host import _signed
    from mpcium_amd.mpcx import ints_to_words, nwords, words_to_ints
    Mw, mn = _signed(ms)
    Rw = ints_to_words(rs, max(nwords(r) for r in rs))
    Bw, bn = _signed(bs)
    cn0 = np.zeros(batch, dtype=np.uint8)
    _kernel_stats_reset()
    t0 = time.perf_counter()
    for _ in range(reps):
        cw, e1 = pk.encrypt_words(Mw, mn, Rw)
        ow, e2 = pk.homo_mult_words(Bw, bn, cw, cn0)
    el_seq = time.perf_counter() - t0
    if e1.any() or e2.any():
        raise SystemExit("paillier line: error codes (timed loop)")
    cs_t, out_t = words_to_ints(cw), words_to_ints(ow)
    for i in range(0, batch, max(1, batch // 8)):  # the timed loop's last outputs vs the oracle formulas
        if cs_t[i] != gm.paillier_encrypt(N, ms[i], rs[i]) or out_t[i] != gm.paillier_homo_mult(N, bs[i], cs_t[i]):
            raise SystemExit(f"paillier line: timed-loop mismatch at {i}")
    seq_roof = _kernel_roofline()
    # a second, separately labelled shape: `inflight` such batches at once from
    # their own threads (a node's concurrent sessions; the Engine coalesces their
    # launches). Every batch is still 1,024 ops; worker errors fail the run and
    # one worker's last outputs are checked against the oracle formulas.
    inflight = max(1, inflight)
    errors, last = [], {}

    def worker(k):
        try:
            for _ in range(reps):
                c, e1 = pk.encrypt_words(Mw, mn, Rw)
                o, e2 = pk.homo_mult_words(Bw, bn, c, cn0)
                if e1.any() or e2.any():
                    raise RuntimeError(f"worker {k}: error codes")
            if k == 0:
                last["c"], last["o"] = words_to_ints(c), words_to_ints(o)
        except BaseException as ex:  # noqa: BLE001 -- reported below
            errors.append(f"{type(ex).__name__}: {ex}")
    if world > 1:
        dist.barrier()
    _kernel_stats_reset()
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(inflight)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    el = time.perf_counter() - t0
    if errors:
        raise SystemExit(f"paillier line: {len(errors)} worker(s) failed: {errors[0]}")
    for i in range(0, batch, max(1, batch // 16)):
        if last["c"][i] != gm.paillier_encrypt(N, ms[i], rs[i]) or \
                last["o"][i] != gm.paillier_homo_mult(N, bs[i], last["c"][i]):
            raise SystemExit(f"paillier line: in-flight worker 0 mismatch at {i}")
    flight_roof = _kernel_roofline()
    if world > 1:
        el, el_seq = max_over_ranks([el, el_seq], world)
    line = {"metric": "tss-lib paillier Encrypt+HomoMult ops/s (config 1: one batch of 1024 ops at a time, 2048-bit N)",
            "value": batch * reps * world / el_seq, "unit": "Encrypt+HomoMult ops/s", "batch": batch,
            "reps": reps, "seconds": el_seq, "n_gpus": world, "scaling": "weak",
            "batches_in_flight": {"batches": inflight, "value": batch * reps * inflight * world / el,
                                  "seconds": el, "kernel_roofline": flight_roof,
                                  "checked": "worker 0's last batch, 64 outputs vs oracle/gomath.py"},
            "note": "host-buffer API end to end (word arrays -> PCIe -> GPU -> back; the Python-int conversions "
                    "are outside the timed loops); Encrypt's Gamma^m is the bit-exact 1 + mN shortcut, r^N a "
                    "shared-exponent GPU batch, c^b per-operand; value: one 1,024-op batch at a time (BASELINE "
                    "configs[0]); batches_in_flight: a different shape, "
                    f"{inflight} such batches concurrently from their own threads",
            "cpu_baseline": None}
    # Go-equivalent work per op (SURVEY.md 8(d) W = (E + E/4) 2 L^2, L = 128 words of N^2): r^N (E = 2048) + c^b
    # (E = bit length of b < q); a 1,024-op batch is a small latency-bound launch pair, not a throughput shape
    L2 = 2 * 128 * 128
    alg = sum((2048 + 512) * L2 + (b.bit_length() + (b.bit_length() + 3) // 4) * L2 for b in bs) * reps
    line["roofline"] = seq_roof
    line["job_roofline"] = _job_roofline(alg, el_seq, world)
    line["job_roofline"]["scope"] = ("end to end (host buffers incl. PCIe; word arrays, no Python-int conversion in "
                                     "the timed loop); batch of 1,024 = latency-bound")
    line["alg_ops_per_op"] = alg / (batch * reps)
    if cpu:
        line["cpu_baseline"] = cpu_baseline_paillier(N, 12.0, info)
    return line


def cpu_baseline_fermat(seconds: float, info: dict):
    """Config 3's work unit on host cores: the 1024-bit Fermat test
    2^(p-1) mod p of tss-lib's Pocklington check, as a Go Exp (C restatement,
    Go's 64-bit Words)."""
    from oracle import crosscheck as cc
    lib = cc.load_c_oracle(64)
    if lib is None:
        return None
    exp = _c_exp_words(lib, 32)

    def make(t):
        import random
        rng = random.Random(23 + t)

        def one():
            p = rng.getrandbits(1024) | 1 | (1 << 1023)
            exp(2, p - 1, p)
        return one

    r1, rn, thr, raw = _one_and_all(make, seconds, info)
    return {"value": rn, "unit": "1024-bit Fermat tests/s", "cores": thr, "kind": "port", "one_core": r1,
            "python_share": _LAST_PYTHON_SHARE[0],
            "all_cores_extrapolated": r1 * info["nproc"],
            "sample": f"{raw[2]} x 2^(p-1) mod p (1024-bit p) in {raw[3]:.1f} s on {thr} threads; "
                      f"oracle/gomodexp.c (64-bit Words)", **info}


def safeprime_line(num: int, seed: int, cpu: bool, info: dict, world: int = 1, rank: int = 0):
    """Config 3 (BASELINE.json): GeneratePreParams' safe-prime search
    (tss-lib candidate stream, GPU sieve + Fermat, GPU Miller-Rabin): `num`
    1024-bit safe primes in stream order. One GPU: the single-stream search.
    world > 1: the stream's batches dealt round-robin to the ranks
    (shard.safe_primes_sharded, same primes as one GPU), strong scaling."""
    from mpcium_amd import host as mhost
    from mpcium_amd.shard import max_over_ranks, safe_primes_sharded
    mhost.init(gpu_index())
    mhost.safe_primes(1024, 1, seed=seed + 1)  # warm-up (allocations, first launches)
    if world > 1:
        import torch.distributed as dist
        acc = {"candidates": 0, "sieved_out": 0, "fermat_tests": 0, "mr_tests": 0, "lucas_tests": 0}

        def fn(b):
            r, s_ = mhost.safe_prime_batch(1024, seed, b)
            for k in acc:
                acc[k] += s_[k]
            return r

        dist.barrier()
        t0 = time.perf_counter()
        sp_stats = {}
        res = safe_primes_sharded(num, rank, world, fn, stats=sp_stats)
        el = time.perf_counter() - t0
        el = max_over_ranks([el], world)[0]
        import torch
        t = torch.tensor([float(acc[k]) for k in acc], dtype=torch.float64)
        dist.all_reduce(t)  # whole-job candidate / test counts (gloo, host tensors)
        st = dict(zip(acc, (int(x) for x in t)))
    else:
        _kernel_stats_reset()
        t0 = time.perf_counter()
        res, st = mhost.safe_primes(1024, num, seed=seed)
        el = time.perf_counter() - t0
        kr = _kernel_roofline()
    for p, q, _ in res:  # untimed: p = 2q + 1, both prime (CPython pow MR spot check)
        if p != 2 * q + 1 or pow(2, p - 1, p) != 1 or pow(3, q - 1, q) != 1 or q.bit_length() != 1023:
            raise SystemExit("safe-prime line: bad prime")
    line = {"metric": f"1024-bit safe primes/s (config 3: GeneratePreParams search, {world} GPU(s))",
            "value": num / el, "unit": "safe primes/s", "safe_primes": num, "seconds": el,
            "fermat_tests_per_s": st["fermat_tests"] / el, "candidates": st["candidates"],
            "sieved_out": st["sieved_out"], "fermat_tests": st["fermat_tests"], "mr_tests": st["mr_tests"],
            "lucas_tests": st.get("lucas_tests", 0),
            "n_gpus": world, "scaling": "strong", "first_index": res[0][2], "last_index": res[-1][2],
            "roofline": _job_roofline((st["fermat_tests"] + st["mr_tests"]) * alg_macs(1024, 1023) / world, el, world),
            "cpu_baseline": None}
    if world > 1:
        line["sharded_gathers"] = sp_stats  # one all-gather per group of rounds (shard.safe_primes_sharded)
    if world == 1:
        # the dominant kernel's own roofline: k_prime2c's Go-equivalent work
        # (2^(p-1) mod p per sieve survivor, 2^d mod q per ride-along q) over
        # its summed launch time (HIP events on its stream)
        pk = [k for k in kr["kernels"] if k["kind"] == "prime2c"]
        if pk and pk[0]["kernel_ms"] > 0:
            k = pk[0]
            ach = k["alg_ops"] / (k["kernel_ms"] / 1e3)
            line["kernel_roofline"] = {"kernel": "k_prime2c", "bound": "valu", "achieved": ach / 1e12,
                                       "peak": PEAK_INT32_NOMINAL / 1e12, "unit": "TOP/s",
                                       "frac": ach / PEAK_INT32_NOMINAL, "launches": k["launches"],
                                       "tests": k["operands"], "kernel_ms": k["kernel_ms"],
                                       "gpu_busy_s_instrumented": kr["gpu_busy_s"]}
    if cpu:
        b = cpu_baseline_fermat(8.0, info)
        if b:
            # host safe-prime rate at the same Fermat tests per safe prime (the Exp dominates tss-lib's loop)
            b["safe_primes_per_s_equiv"] = b["value"] / (st["fermat_tests"] / num)
        line["cpu_baseline"] = b
    return line


def load_nodes():
    with open(os.path.join(ROOT, "tests", "golden", "node_preparams.json")) as f:
        d = json.load(f)
    return [{k: int(v, 16) for k, v in n.items() if isinstance(v, str) and k != "paillier_source"}
            for n in d["nodes"]]


def _signing_worker(args):
    """One process of the signing CPU baseline: whole GG18 signatures of
    `signers` of the fixture nodes, wallet after wallet, until the deadline
    (oracle/signing_ref.py sign_wallet: every ordered pair's MtA / MtAwc with
    all proofs verified, then rounds 1/4-9 and ecdsa.Verify), with Go's expNN
    restated in C (oracle/gomodexp.c, 64-bit Words) and secp256k1 through
    OpenSSL (oracle/ossl_ec.py). Returns (signatures, seconds inside the C
    arithmetic, seconds)."""
    deadline, seed, signers = args
    from oracle import crosscheck as cc
    from oracle import mta_ref as M
    from oracle import ossl_ec
    from oracle import signing_ref as S
    lib = cc.load_c_oracle(64)
    ec = ossl_ec.install()
    c_mod = [0.0]

    def pw(x, y, m):
        t = time.perf_counter()
        r = cc.c_expnn(lib, x % m, y, m)
        c_mod[0] += time.perf_counter() - t
        return r
    M._pw = pw
    nodes = load_nodes()
    t0 = time.perf_counter()
    sigs, wi = 0, 0
    while time.time() < deadline:
        _, sig, ok, _ = S.sign_wallet(nodes, signers, seed, wi)
        if not ok:
            raise SystemExit("signing CPU baseline: a signature did not verify")
        wi += 1
        if time.time() <= deadline:
            sigs += 1
    return sigs, c_mod[0] + ec.c_seconds, time.perf_counter() - t0


def _keygen_worker(args):
    """One process of the config-5 CPU baseline: cycles through the six proof
    primitives (oracle/proofs_ref.py with Go's expNN restated in C) until the
    deadline; returns {primitive: [count, seconds]}."""
    deadline, seed = args
    from oracle import crosscheck as cc
    from oracle import proofs_ref as PR
    from oracle import safeprime_ref as SP
    from oracle import tss_ref as T
    lib = cc.load_c_oracle(64)
    c_s = [0.0]

    def pw(x, y, m):
        t = time.perf_counter()
        r = cc.c_expnn(lib, x % m, y, m)
        c_s[0] += time.perf_counter() - t
        return r
    PR._pw = SP._pw = pw
    t_start = time.perf_counter()
    nodes = load_nodes()
    A, B = nodes[0], nodes[1]
    rd = T.Reader(seed)
    ss = rd.read(32)
    acc = {k: [0, 0.0] for k in ("dln_prove", "dln_verify", "mod_prove", "mod_verify", "fac_prove", "fac_verify")}
    dln = mod = fac = None
    while time.time() < deadline:
        t = time.perf_counter()
        dln = PR.dln_prove(A["H1i"], A["H2i"], A["Alpha"], A["p"], A["q"], A["NTildei"], rd)
        acc["dln_prove"][0] += 1
        acc["dln_prove"][1] += time.perf_counter() - t
        t = time.perf_counter()
        assert PR.dln_verify(dln, A["H1i"], A["H2i"], A["NTildei"])
        acc["dln_verify"][0] += 1
        acc["dln_verify"][1] += time.perf_counter() - t
        t = time.perf_counter()
        mod = PR.mod_prove(ss, A["N"], A["P"], A["Q"], rd)
        acc["mod_prove"][0] += 1
        acc["mod_prove"][1] += time.perf_counter() - t
        t = time.perf_counter()
        assert PR.mod_verify(mod, ss, A["N"])
        acc["mod_verify"][0] += 1
        acc["mod_verify"][1] += time.perf_counter() - t
        t = time.perf_counter()
        fac = PR.fac_prove(ss, A["N"], B["NTildei"], B["H1i"], B["H2i"], A["P"], A["Q"], rd)
        acc["fac_prove"][0] += 1
        acc["fac_prove"][1] += time.perf_counter() - t
        t = time.perf_counter()
        assert PR.fac_verify(fac, ss, A["N"], B["NTildei"], B["H1i"], B["H2i"])
        acc["fac_verify"][0] += 1
        acc["fac_verify"][1] += time.perf_counter() - t
    acc["_c_seconds"] = [0, c_s[0]]
    acc["_seconds"] = [0, time.perf_counter() - t_start]
    return acc


def cpu_baseline_keygen(seconds: float, info: dict, parties: int):
    """Config 5 on host cores: per-primitive times of the proof restatement
    (one process per core, all running at once), composed into the per-session
    mix of keygenload.hpp: n(2 DLN + Mod + (n-1) Fac) proofs and
    n(n-1)(2 DLN + Mod + Fac) verifications."""
    from concurrent.futures import ProcessPoolExecutor
    import multiprocessing as mp
    from oracle import crosscheck as cc
    if cc.load_c_oracle(64) is None:
        return None
    procs = info["usable_threads"]
    deadline = time.time() + seconds
    with ProcessPoolExecutor(procs, mp_context=mp.get_context("fork")) as ex:
        res = list(ex.map(_keygen_worker, [(deadline, 0x6B0 + i) for i in range(procs)]))
    c_share = sum(r["_c_seconds"][1] for r in res) / max(1e-9, sum(r["_seconds"][1] for r in res))
    tot = {k: [sum(r[k][0] for r in res), sum(r[k][1] for r in res)] for k in res[0] if not k.startswith("_")}
    if any(c == 0 for c, _ in tot.values()):
        return None
    per = {k: s / c for k, (c, s) in tot.items()}
    n = parties
    mix = {"dln_prove": 2 * n, "mod_prove": n, "fac_prove": n * (n - 1),
           "dln_verify": 2 * n * (n - 1), "mod_verify": n * (n - 1), "fac_verify": n * (n - 1)}
    cpu_s = sum(mix[k] * per[k] for k in mix)
    return {"value": procs / cpu_s, "unit": "sessions/s", "cores": procs, "kind": "port",
            "one_core": 1.0 / cpu_s, "all_cores_extrapolated": info["nproc"] / cpu_s,
            "per_primitive_s": per, "python_share": 1.0 - c_share, **info,
            "sample": f"{sum(c for c, _ in tot.values())} proof primitives (DLN/Mod/Fac prove + verify) in "
                      f"{seconds:.0f} s on {procs} processes, composed into one {n}-party session's mix "
                      f"({cpu_s:.1f} CPU-s per session); oracle/proofs_ref.py with Go expNN restated in C "
                      f"(64-bit Words); python_share = time outside those C calls (the Lucas test and "
                      f"Jacobi symbols run in Python); one_core = 1 / CPU-s per session"}


def keygen_line(args, world: int = 1, rank: int = 0):
    """Config 5 (BASELINE.json): keygen / reshare proof work under load --
    every party of every session proves DLN x2 + Mod + Fac per peer and
    verifies all peers' proofs (csrc/host/keygenload.hpp), 5 parties (3-of-5),
    on one GPU. Parties: the 3 fixture nodes plus 2 generated here by the GPU
    GeneratePreParams (untimed). world > 1: every rank runs its own
    `keygen_sessions` sessions (weak scaling); value = all ranks' sessions /
    max time."""
    from mpcium_amd import host as mhost
    from mpcium_amd import proofs as mproofs
    mhost.init(gpu_index())
    parties = load_nodes()
    for seed in (0x6D706335, 0x6D706336)[:max(0, args.parties - len(parties))]:
        pp, _ = mhost.generate_preparams(seed=seed)
        parties.append(pp)
    parties = parties[:args.parties]
    # warm-up of one wave: the node-lifetime fixed-base comb tables (h1, h2 of
    # every party's N~ and their inverses) are built on first use, as a node
    # builds them once for its peers' preparams, not per session
    wave = args.keygen_wave or 1024
    mixed = bool(args.reshare_mix)
    # (two waves when mixed: the resharing wave's EC paths warm up too)
    warm = mproofs.bench_keygen_proofs(parties, min(wave * (2 if mixed else 1), args.keygen_sessions), seed=0x6B66,
                                       wave=wave, reshare=mixed)
    if warm["failures"] or warm.get("vss_failures"):
        raise SystemExit(f"keygen proofs warmup: {warm}")
    import resource
    rss0 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    _kernel_stats_reset()
    if world > 1:
        import torch.distributed as dist
        from mpcium_amd.shard import max_over_ranks
        dist.barrier()
    st = mproofs.bench_keygen_proofs(parties, args.keygen_sessions, seed=0x6B67 + 7919 * rank, wave=wave,
                                     reshare=mixed)
    rss1 = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss
    if st["failures"] or st.get("vss_failures"):
        raise SystemExit(f"rank {rank}: keygen proofs: {st}")
    total_s = st["total_s"]
    if world > 1:
        total_s = max_over_ranks([total_s], world)[0]
    kind = ("keygen + resharing waves alternating (resharing: the new committee's proofs + the old committee's VSS, "
            "mpcium's two sessions per node)" if mixed else "keygen waves only")
    line = {"metric": f"{len(parties)}-party keygen/reshare sessions/s (config 5: DLN x2 + Mod + Fac proofs per party, "
                      f"every peer verified, {args.keygen_sessions} sessions, {kind})",
            "value": st["sessions"] * world / total_s, "unit": "sessions/s", "n_gpus": world, "scaling": "weak",
            "concurrent_sessions": min(int(st["sessions"]), 2 * wave),
            "host_rss_gb": rss1 / 1024.0 / 1024.0,
            "sessions": int(st["sessions"]), "parties": len(parties), "proofs": int(st["proofs"]),
            "verifications": int(st["verifications"]), "seconds": st["total_s"], "prove_s": st["prove_s"],
            "verify_s": st["verify_s"], "engine_busy_s": st["engine_busy_s"],
            "waves": int(st["waves"]), "wave_sessions": int(st["wave_sessions"]), "max_wave_s": st["max_wave_s"],
            "host_max_rss_mb": rss1 / 1024.0, "host_max_rss_mb_before": rss0 / 1024.0,
            "verifications_per_s": st["verifications"] * world / total_s, "checked": "every verification passes",
            "concurrency_note": "sessions stream in waves of wave_sessions, two waves in flight: at most "
                                "2 x wave_sessions sessions are concurrent (measured faster than larger waves, "
                                "DESIGN.md 6)",
            "roofline": _kernel_roofline(),
            "job_roofline": _job_roofline(st["alg_macs"], total_s, world),
            "cpu_baseline": None}
    if mixed:
        # each kind's sessions over the time its waves were running (the two
        # kinds share the GPU the whole time, so each is a rate within the mix)
        ks, rs = st["keygen_sessions"], st["reshare_sessions"]
        line["keygen_sessions"], line["reshare_sessions"] = int(ks), int(rs)
        line["keygen_value"] = ks * world / total_s
        line["reshare_value"] = rs * world / total_s
        line["keygen_wave_s_mean"] = st["keygen_wave_s"] / max(1, (st["waves"] + 1) // 2)
        line["reshare_wave_s_mean"] = st["reshare_wave_s"] / max(1, st["waves"] // 2)
        line["vss_checks"], line["vss_failures"] = int(st["vss_checks"]), int(st["vss_failures"])
        line["rates_note"] = ("keygen_value / reshare_value: each kind's sessions over the whole run (the kinds' waves "
                              "alternate and share the GPU; value = their sum); *_wave_s_mean: one wave of that kind "
                              "(wave_sessions sessions) while the other kind's wave runs beside it")
    return line


def cpu_baseline_signing(seconds: float, info: dict, signers: int):
    """GG18 signing on host cores: the oracle restatement of tss-lib's signing
    (MtA / MtAwc with range proofs, rounds 1/4-9, ecdsa.Verify) with its
    arithmetic in C -- Go's expNN restated (oracle/gomodexp.c) and OpenSSL
    secp256k1 -- one process per usable core. python_share: the part of the
    processes' time outside those C calls (Python orchestration, hashing,
    draws), which a Go build would spend in Go."""
    from concurrent.futures import ProcessPoolExecutor
    from oracle import crosscheck as cc
    if cc.load_c_oracle(64) is None:
        return None
    procs = info["usable_threads"]
    t0 = time.time()
    deadline = t0 + seconds
    import multiprocessing as mp
    with ProcessPoolExecutor(procs, mp_context=mp.get_context("fork")) as ex:
        res = list(ex.map(_signing_worker, [(deadline, 0x51C0 + 97 * i, signers) for i in range(procs)]))
    el = max(time.time() - t0, seconds)
    n = sum(r[0] for r in res)
    c_s, tot_s = sum(r[1] for r in res), sum(r[2] for r in res)
    return {"value": n / el, "unit": "sigs/s", "cores": procs, "kind": "port", "signers": signers,
            "one_core": n / el / procs, "all_cores_extrapolated": n / el / procs * info["nproc"],
            "python_share": 1.0 - c_s / max(tot_s, 1e-9), **info,
            "sample": f"{n} whole {signers}-signer GG18 signatures (every ordered pair's MtA/MtAwc with all "
                      f"proofs verified, rounds 1/4-9 commitments and Schnorr/ZKV proofs, ecdsa.Verify) in "
                      f"{el:.1f} s on {procs} processes; oracle/signing_ref.py with Go expNN restated in C "
                      f"(oracle/gomodexp.c, 64-bit Words) and OpenSSL secp256k1 (oracle/ossl_ec.py); "
                      f"python_share = time outside those C calls; one_core = per process while all ran"}


def _job_roofline(alg_macs: float, seconds: float, world: int = 1) -> dict:
    """Whole-job roofline of a protocol line: the Go-equivalent algorithmic
    work the host mirror sent to the GPU (Engine::alg_macs, SURVEY.md 8(d) W
    per exponentiation) over the line's wall time, against the nominal INT32
    MAD peak of the GPUs. Host-side work (hashing, draws, gcds, packing) is in
    the wall time, so this is an end-to-end figure, not a kernel roofline."""
    achieved = alg_macs * world / seconds
    return {"bound": "valu", "achieved": achieved / 1e12, "peak": PEAK_INT32_NOMINAL * world / 1e12,
            "unit": "TOP/s", "frac": achieved / (PEAK_INT32_NOMINAL * world), "traffic": None,
            "alg_ops_per_job": alg_macs, "scope": "end to end (wall time incl. host work)",
            "note": "alg_ops are Go-equivalent (SURVEY.md 8(d) W per Exp, Go's 4-bit window); the GPU does less "
                    "real work for the same Exps (fixed-base comb tables, CRT, sliding windows, algebraic "
                    "shortcuts), so this job-level ratio can exceed 1: a rate of Go-equivalent work, not a "
                    "utilization"}


def _kernel_stats_reset():
    """Start per-kernel GPU timing (mpcx_kernel_stats) for a protocol line's
    timed region: an event pair around every launch, read at the lane's
    host wait (a few us per launch of several ms)."""
    from mpcium_amd import mpcx
    mpcx.set_option("kernel_stats", 1)
    mpcx.kernel_stats(reset=True)


def _kernel_roofline(world: int = 1) -> dict:
    """Kernel-level roofline of a protocol line (VALU-bound big-int kernels):
    the kernels' work MACs over the GPU busy time -- the union of every
    launch's [start, end) on the device, so overlapping lanes count once --
    against the nominal INT32 MAD peak. Work MACs: Go-equivalent W for the
    exponentiation kernels (within ~5% of executed: same squarings, 5-bit /
    sliding windows), executed products x 2 L^2 for the fixed-base comb.
    Per kernel: its MACs over its summed launch durations (concurrent lanes
    share the CUs, so these understate each kernel in isolation)."""
    from mpcium_amd import mpcx
    ks = mpcx.kernel_stats()
    mpcx.set_option("kernel_stats", 0)
    busy_s = ks["busy_ms"] / 1e3
    tot_ms = sum(k["kernel_ms"] for k in ks["kernels"]) or 1e-9
    per = []
    for k in sorted(ks["kernels"], key=lambda k: -k["kernel_ms"]):
        t = k["kernel_ms"] / 1e3
        per.append({"kind": k["kind"], "geom": k["geom"], "launches": k["launches"], "operands": k["operands"],
                    "kernel_ms": k["kernel_ms"], "share_of_kernel_time": k["kernel_ms"] / tot_ms,
                    "alg_ops": k["alg_macs"],
                    "frac": (k["alg_macs"] / t / PEAK_INT32_NOMINAL) if t > 0 and k["alg_macs"] else None})
    ach = ks["alg_macs"] / busy_s if busy_s > 0 else 0.0
    return {"bound": "valu", "achieved": ach / 1e12, "peak": PEAK_INT32_NOMINAL / 1e12, "unit": "TOP/s",
            "frac": ach / PEAK_INT32_NOMINAL, "traffic": None, "gpu_busy_s": busy_s, "world": world,
            "scope": "GPU busy time of rank 0's device (union of launch intervals), all kernels' work MACs",
            "kernels": per}


def signing_line(args, world, rank, signers: int):
    """Config 4 (BASELINE.json): GG18 ECDSA signing of `wallets` wallets per
    GPU by `signers` of the 3 nodes (csrc/host/signing.hpp): MtA / MtAwc with
    range proofs on the GPU, then delta, sigma, R, s and ecdsa.Verify of every
    signature (/root/reference/pkg/mpc/ecdsa_signing_session.go:162). Each rank
    signs its own wallets (weak scaling); value = all ranks' verified
    signatures / max time."""
    import torch
    import torch.distributed as dist
    from mpcium_amd import host as mhost
    from mpcium_amd import mta
    from mpcium_amd.shard import max_over_ranks
    mhost.init(gpu_index())
    nodes = load_nodes()
    # warm-up at the timed size: lane staging buffers and workspaces reach
    # their steady-state sizes (a node's steady state), so the timed run does
    # no hipMalloc / hipFree
    warm = mta.bench_signing(nodes, signers, args.wallets, seed=0x5167 + 7919 * rank)
    if warm["errors"] or warm["relation_failures"] or warm["verified"] != args.wallets:
        raise SystemExit(f"rank {rank}: signing warmup failed: {warm}")
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    mhost.profile_report(reset=True)
    _kernel_stats_reset()
    import resource
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    t0 = time.perf_counter()
    st = mta.bench_signing(nodes, signers, args.wallets, seed=0x5168 + 7919 * rank)
    torch.cuda.synchronize()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    host_cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if st["errors"] or st["relation_failures"] or st["verified"] != args.wallets or st["aborted"]:
        raise SystemExit(f"rank {rank}: signing failed: {st}")
    el, r1, r2, r3, fin = max_over_ranks([el, st["round1_s"], st["round2_s"], st["round3_s"], st["finalize_s"]],
                                         world)
    line = {"metric": f"{signers}-of-3 ECDSA sigs/s over {args.wallets * world // 1000}k wallets "
                      f"(GG18 signing, every Paillier/DLN exponentiation on the GPU, every signature verified)",
            "value": args.wallets * world / el, "unit": "sigs/s", "n_gpus": world,
            "wallets_per_gpu": args.wallets, "signers": signers, "seconds": el,
            "signatures_verified": int(st["verified"]) * world,
            "rounds_s": {"round1_alice_init": r1, "round2_bob_mid": r2, "round3_alice_end": r3,
                         "rounds4_9_finalize_verify": fin},
            "host_cpu_s_per_signature": host_cpu_s / args.wallets,
            "engine_busy_s": st["engine_busy_s"], "host_share": 1.0 - st["engine_busy_s"] / max(el, 1e-9),
            "host_cpu_s": host_cpu_s,
            "sessions_per_gpu": int(st["sessions"]),
            "checked": "alpha+beta == k*gamma, mu+nu == k*w (mod q) on every session; every round-1/4-9 "
                       "commitment, Schnorr and ZKV proof of every signer; ecdsa.Verify of every signature by "
                       "every signer (tss-lib finalize and mpcium's session)",
            "roofline": _kernel_roofline(world),
            "job_roofline": _job_roofline(st["alg_macs"], el, world),
            "alg_ops_per_signature": st["alg_macs"] / args.wallets,
            "scope": "all of tss-lib's GG18 signing rounds: MtA/MtAwc + range proofs (rounds 1-3) on the GPU; "
                     "round-1/5/7 commitments, round-4/6 Schnorr and ZKV proofs and their verification, "
                     "finalize and ecdsa.Verify on the host",
            "cpu_baseline": None}
    prof = mhost.profile_report()
    if prof:  # MPCX_HOST_PROFILE=1: host seconds per label, summed over threads
        line["host_profile"] = prof.strip().splitlines()
    return line


LINE_MAX_BYTES = 4096  # the driver keeps a bounded tail of stdout: the result line must fit in it whole

# sub-line key of the detail dict -> short key in the printed line
_SUBLINES = (("paillier_batch", "c1_paillier"), ("safe_prime", "c3_safe_primes"), ("signing", "c4_sign"),
             ("signing_3_signers", "c4_sign_3_signers"), ("keygen", "c5_keygen"))


def _r(x, nd=4):
    """Round a float to `nd` significant digits (None passes through)."""
    if x is None or not isinstance(x, float):
        return x
    return float(f"{x:.{nd}g}")


def compact_line(result: dict, detail_path: str | None) -> dict:
    """The ONE line bench.py prints: the contract keys, the headline roofline
    and cpu_baseline, and per config {value, unit, frac, cpu, cores}. Every
    other field (per-step times, telemetry, per-kernel lists, samples, notes,
    host profiles) stays in the detail file the line names. Guaranteed to
    serialise to at most LINE_MAX_BYTES (tests/test_bench_line.py)."""
    keep = ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
            "vs_baseline", "dtype")
    line = {k: _r(result.get(k), 6) for k in keep}
    line["data"] = "synthetic (seeded bases < N^2; N = tests/golden/paillier_key_2048.json)"
    c = result.get("config") or {}
    line["config"] = {k: c.get(k) for k in ("workload", "operands_per_gpu", "modulus_bits", "exp_bits",
                                             "parallelism") if k in c}
    r = result.get("roofline") or {}
    line["roofline"] = {"bound": r.get("bound"), "achieved": _r(r.get("achieved")), "peak": _r(r.get("peak")),
                        "unit": r.get("unit"), "frac": _r(r.get("frac")), "traffic": r.get("traffic"),
                        "kernel_ms": _r(r.get("kernel_ms"), 5)}
    if r.get("frac_at_measured_clock") is not None:
        line["roofline"]["frac_at_clock"] = _r(r["frac_at_measured_clock"])
    if r.get("frac_at_clock") is not None:
        line["roofline"]["frac_at_clock"] = _r(r["frac_at_clock"])
    if r.get("kernel"):
        line["roofline"]["kernel"] = r["kernel"]
    if r.get("go_equiv_frac") is not None:
        # two-pipe kernel (two_pipe_roofline): frac is the executed-work floor's; the
        # Go-equivalent INT32 ratio and the matrix pipe's rate sit beside it
        for k in ("binding_pipe", "peak_i8", "achieved_i8", "frac_i8", "go_equiv_frac", "go_equiv_achieved"):
            line["roofline"][k] = _r(r[k]) if isinstance(r.get(k), float) else r.get(k)
    cb = result.get("cpu_baseline")
    line["cpu_baseline"] = None if not cb else {
        "value": _r(cb.get("value")), "unit": cb.get("unit"), "cores": cb.get("cores"), "kind": cb.get("kind"),
        "sample": "Go expNNMontgomery restated in C (64-bit Words), x^N mod N^2 on the host's usable threads"}
    dg = result.get("batch_digest")
    if dg is not None:
        line["digest_match"] = bool(dg.get("match"))
    cfg = {}
    po = result.get("config2_per_operand_exponents") or []
    for s in po:
        cfg[f"c2_per_op_{s['exp_bits']}"] = {"value": _r(s.get("value")), "unit": s.get("unit"),
                                             "frac": _r((s.get("roofline") or {}).get("frac"), 3)}
    for src, dst in _SUBLINES:
        s = result.get(src)
        if not s:
            continue
        fr = (s.get("kernel_roofline") or s.get("roofline") or {}).get("frac")
        sb = s.get("cpu_baseline") or {}
        cpu = sb.get("safe_primes_per_s_equiv", sb.get("value"))  # config 3: in the line's own unit
        cfg[dst] = {"value": _r(s.get("value")), "unit": s.get("unit"), "n_gpus": s.get("n_gpus"),
                    "frac": _r(fr, 3), "cpu": _r(cpu), "cores": sb.get("cores")}
        bif = s.get("batches_in_flight")
        if isinstance(bif, dict):  # config 1's second shape, labelled
            cfg[dst]["batches_in_flight"] = bif.get("batches")
            cfg[dst]["in_flight_value"] = _r(bif.get("value"))
        for k in ("sessions", "concurrent_sessions", "reshare_value", "keygen_value", "host_rss_gb"):
            if s.get(k) is not None:
                cfg[dst][k] = _r(s[k]) if isinstance(s[k], float) else s[k]
    line["configs"] = cfg
    line["detail"] = detail_path
    # last resort: never exceed the driver's tail (drop the configs, which are in the detail file)
    if len(json.dumps(line)) > LINE_MAX_BYTES:
        line["configs"] = {k: {"value": v["value"], "unit": v["unit"]} for k, v in cfg.items()}
    if len(json.dumps(line)) > LINE_MAX_BYTES:
        line.pop("configs")
    return line


def node_main(args, progress) -> None:
    """--node: mpcium's deployment shape -- ONE process per node drives every
    GPU of the node (/root/reference/cmd/mpcium/main.go:150,
    /root/reference/pkg/mpc/node.go:59-88: one preparams set shared by every
    wallet session of the node). libmpcx binds the devices with
    mpcx_init_devices; config 2 runs one resident batch per device, launched
    from this one process onto each device's stream; configs 4 and 5 run
    through the one Engine (libmpcx_host), whose batches spread over the
    devices (split batches above device_split_min, round-robin otherwise).
    Work per device is fixed (weak scaling): wallets and sessions scale with
    the device count. --node-dup K rehearses K logical devices on one HIP
    ordinal (mpcx_set_option "duplicate_device"): the node path end to end on a
    one-GPU box, NOT a scaling measurement (the logical devices share one GPU).
    Prints one JSON line (mode "node")."""
    import torch
    from mpcium_amd import host as mhost
    from mpcium_amd import mpcx, mta, proofs as mproofs
    if args.node_dup:
        mpcx.set_option("duplicate_device", 1)
        for _ in range(args.node_dup):
            mhost.init(0)
    else:
        mhost.init_devices(args.node_devices)
    devs = mpcx.bound_devices()
    D = len(devs)
    progress(f"node: {D} bound devices {devs}")
    N = load_key()
    N2 = N * N
    mod = mpcx.Modulus(N2)
    words, count = mod.words, args.count
    exp = mpcx.int_to_words(N, mpcx.nwords(N))
    L = mpcx.lib()
    per = []
    for d, ordinal in enumerate(devs):
        dev = torch.device("cuda", ordinal)
        bases = synth_bases(N2, count, 0x6D706332 + d, words)
        per.append({"d": d, "dev": dev, "bases": bases, "st": torch.cuda.Stream(dev),
                    "b": torch.from_numpy(bases.view(np.int32)).to(dev),
                    "e": torch.from_numpy(exp.view(np.int32)).to(dev),
                    "o": torch.zeros((count, words), dtype=torch.int32, device=dev)})

    def launch(p):
        mpcx.select_device(p["d"])
        with torch.cuda.device(p["dev"]):
            rc = L.mpcx_modexp_batch_device(mod.handle, count, p["b"].data_ptr(), words, p["e"].data_ptr(),
                                            len(exp), 1, N.bit_length(), p["o"].data_ptr(), words,
                                            p["st"].cuda_stream)
        if rc != 0:
            raise mpcx.MpcxError(rc, L.mpcx_last_error().decode())

    def sync_all():
        for p in per:
            p["st"].synchronize()

    progress("node: config 2 warm-up")
    for _ in range(args.warmup):
        for p in per:
            launch(p)
    sync_all()
    l0 = [mpcx.device_launches(d) for d in range(D)]
    for p in per:
        p["ev"] = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    t0 = time.perf_counter()
    for p in per:
        p["ev"][0].record(p["st"])
    for _ in range(args.steps):  # every device's launches queued from this one thread
        for p in per:
            launch(p)
    for p in per:
        p["ev"][1].record(p["st"])
    sync_all()
    el = time.perf_counter() - t0
    kms = [p["ev"][0].elapsed_time(p["ev"][1]) / max(1, args.steps) for p in per]
    launches = [mpcx.device_launches(d) - l0[d] for d in range(D)]
    bad = []
    for p in per:  # untimed: sampled outputs of every device against pow()
        out = p["o"].cpu().numpy().view(np.uint32)
        idx = np.linspace(0, count - 1, max(2, args.verify)).astype(int)
        xs, zs = mpcx.words_to_ints(p["bases"][idx]), mpcx.words_to_ints(out[idx])
        bad += [(p["d"], int(i)) for i, x, z in zip(idx, xs, zs) if pow(x, N, N2) != z]
    if bad:
        raise SystemExit(f"node: config-2 results differ from pow() at {bad[:5]}")
    digest = None
    gd_path = os.path.join(ROOT, "tests", "golden", "batch_digest.json")
    if os.path.exists(gd_path):
        gd = json.load(open(gd_path))
        if gd["count"] == count and gd["words"] == words and args.steps + args.warmup > 0:
            import hashlib
            got = hashlib.sha256(per[0]["o"].cpu().numpy().astype("<u4").tobytes()).hexdigest()
            digest = {"match": got == gd["sha256"], "scope": "device 0's batch vs the C restatement"}
            if not digest["match"]:
                raise SystemExit("node: device 0 batch digest differs from the C restatement")
    W = alg_macs(N2.bit_length(), N.bit_length())
    result = {"metric": METRIC, "mode": "node", "value": count * D * args.steps / el, "unit": "modexp/s",
              "n_gpus": D, "steps": args.steps, "warmup": args.warmup, "ms_per_step": el / max(1, args.steps) * 1e3,
              "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
              "data": "synthetic (seeded bases < N^2 per device; N = tests/golden/paillier_key_2048.json)",
              "config": {"workload": "config2: x^N mod N^2, 4096-bit modulus, shared 2048-bit exponent y=N",
                         "operands_per_gpu": count, "parallelism": f"node process x {D} devices (no collective)",
                         "devices": devs, "duplicated_ordinal_rehearsal": bool(args.node_dup)},
              "roofline": {"bound": "valu", "unit": "TOP/s", "peak": PEAK_INT32_NOMINAL / 1e12,
                           "achieved": W * count / (max(kms) * 1e-3) / 1e12,
                           "frac": W * count / (max(kms) * 1e-3) / PEAK_INT32_NOMINAL, "traffic": None,
                           "kernel_ms_per_device": kms},
              "device_launches": {"config2": launches}, "cpu_baseline": None}
    if mpcx.get_option("mx") == 1 and count >= mpcx.get_option("mx_min"):
        # the same two-pipe roofline as the per-rank line, per device
        result["roofline"]["kernel_ms"] = max(kms)
        result["roofline"]["kernel"] = "k_modexp_mx"
        result["roofline"]["executed_floor"] = mx_floor(count, N, max(kms))
        two_pipe_roofline(result["roofline"])
    if digest:
        result["batch_digest"] = digest
    nodes = load_nodes()
    if args.wallets > 0:
        progress(f"node: config 4 signing, {args.wallets * D} wallets over {D} devices")
        wl = args.wallets * D
        warm = mta.bench_signing(nodes, args.signers, wl, seed=0x5167)
        if warm["errors"] or warm["verified"] != wl:
            raise SystemExit(f"node: signing warm-up failed: {warm}")
        l1 = [mpcx.device_launches(d) for d in range(D)]
        _kernel_stats_reset()
        t1 = time.perf_counter()
        st = mta.bench_signing(nodes, args.signers, wl, seed=0x5168)
        e1 = time.perf_counter() - t1
        if st["errors"] or st["relation_failures"] or st["verified"] != wl or st["aborted"]:
            raise SystemExit(f"node: signing failed: {st}")
        result["signing"] = {"value": wl / e1, "unit": "sigs/s", "n_gpus": D, "wallets": wl, "seconds": e1,
                             "signatures_verified": int(st["verified"]),
                             "device_launches": [mpcx.device_launches(d) - l1[d] for d in range(D)],
                             "roofline": _kernel_roofline(D)}
    if args.keygen_sessions > 0:
        parties = nodes
        for seed in (0x6D706335, 0x6D706336)[:max(0, args.parties - len(parties))]:
            pp, _ = mhost.generate_preparams(seed=seed)
            parties.append(pp)
        parties = parties[:args.parties]
        ks = args.keygen_sessions * D
        wave = args.keygen_wave or 1024
        progress(f"node: config 5, {ks} keygen/reshare sessions over {D} devices")
        mixed = bool(args.reshare_mix)
        warm = mproofs.bench_keygen_proofs(parties, min(ks, wave * 2), seed=0x6B66, wave=wave, reshare=mixed)
        if warm["failures"] or warm.get("vss_failures"):
            raise SystemExit(f"node: keygen warm-up failed: {warm}")
        l2 = [mpcx.device_launches(d) for d in range(D)]
        _kernel_stats_reset()
        st = mproofs.bench_keygen_proofs(parties, ks, seed=0x6B67, wave=wave, reshare=mixed)
        if st["failures"] or st.get("vss_failures"):
            raise SystemExit(f"node: keygen failed: {st}")
        result["keygen"] = {"value": st["sessions"] / st["total_s"], "unit": "sessions/s", "n_gpus": D,
                            "sessions": int(st["sessions"]), "seconds": st["total_s"],
                            "reshare_sessions": int(st.get("reshare_sessions", 0)),
                            "device_launches": [mpcx.device_launches(d) - l2[d] for d in range(D)],
                            "roofline": _kernel_roofline(D)}
    progress("node: done")
    detail = os.path.abspath(args.detail)
    os.makedirs(os.path.dirname(detail), exist_ok=True)
    with open(detail, "w") as f:
        json.dump(result, f, indent=1)
    line = {k: result[k] for k in ("metric", "mode", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
                                   "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config")}
    line["roofline"] = {k: _r(v) if isinstance(v, float) else v for k, v in result["roofline"].items()
                        if k not in ("kernel_ms_per_device", "executed_floor", "go_equiv_note")}
    line["cpu_baseline"] = None
    line["device_launches"] = result["device_launches"]["config2"]
    if digest:
        line["digest_match"] = digest["match"]
    for k, dst in (("signing", "c4_sign"), ("keygen", "c5_keygen")):
        if k in result:
            line.setdefault("configs", {})[dst] = {"value": _r(result[k]["value"]), "unit": result[k]["unit"],
                                                   "n_gpus": D, "device_launches": result[k]["device_launches"]}
    line["detail"] = os.path.relpath(detail, ROOT)
    print(json.dumps(line), flush=True)


def relaunch_under_torchrun(args, argv) -> int:
    """--gpus N > 1 without a launcher: start torchrun with N local ranks as a
    CHILD process (nothing in this process has touched the GPU yet) and return
    its exit code; rank 0 of the child prints the line."""
    import socket
    import subprocess
    with socket.socket() as s:  # a free port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    print(f"[bench] --gpus {args.gpus} without WORLD_SIZE: running {' '.join(cmd)}", file=sys.stderr, flush=True)
    return subprocess.call(cmd)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--count", type=int, default=65536, help="operands per GPU per step")
    ap.add_argument("--cpu-seconds", type=float, default=20.0)
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-smi", action="store_true", help="no amdsmi clock/power sampler beside the timed steps")
    ap.add_argument("--verify", type=int, default=16, help="results checked against CPython pow (untimed)")
    ap.add_argument("--opt", action="append", default=[], help="libmpcx tuning knob key=value (mpcx_set_option)")
    ap.add_argument("--wallets", type=int, default=10000,
                    help="config 4: wallets per GPU for the 2-of-3 signing MtA line (0: skip)")
    ap.add_argument("--signers", type=int, default=2)
    ap.add_argument("--no-sign3", action="store_true", help="skip the 3-signer signing line (timeline runs)")
    ap.add_argument("--keygen-sessions", type=int, default=50000,
                    help="config 5: keygen/reshare sessions for the proof-work line (0: skip)")
    ap.add_argument("--keygen-wave", type=int, default=0,
                    help="config 5: sessions per bounded-memory wave (0: the driver's 1024)")
    ap.add_argument("--parties", type=int, default=5)
    ap.add_argument("--reshare-mix", type=int, default=1,
                    help="config 5: 1 -- alternate keygen and resharing waves (mpcium's old + new party sessions); "
                         "0 -- keygen waves only")
    ap.add_argument("--paillier-inflight", type=int, default=16,
                    help="config 1: batches of 1,024 in flight from their own threads (concurrent sessions)")
    ap.add_argument("--extra-lines", type=int, default=1,
                    help="1: add the config-1 (Paillier batch) and config-3 (safe primes) objects at N=1")
    ap.add_argument("--cpu-sign-seconds", type=float, default=15.0)
    ap.add_argument("--safe-primes", type=int, default=256,
                    help="config 3: 1024-bit safe primes to find (256: steady state, ~4 steps per GPU at N = 8)")
    ap.add_argument("--modbits", type=int, default=4096, choices=(2048, 4096),
                    help="4096: x^N mod N^2 (config 2, the bench line); 2048: x^N mod N (Paillier N / N~ class)")
    ap.add_argument("--detail", default=os.path.join("gpurun_out", "bench_detail.json"),
                    help="file for the full result (per-step times, telemetry, per-kernel lists, samples); "
                         "the printed line names it")
    ap.add_argument("--node", action="store_true",
                    help="one process drives every GPU of the node (mpcium's shape; see node_main)")
    ap.add_argument("--node-devices", type=int, default=0, help="--node: GPUs to bind (0: all visible)")
    ap.add_argument("--node-dup", type=int, default=0,
                    help="--node rehearsal: bind HIP ordinal 0 this many times as logical devices")
    args = ap.parse_args()
    if args.node:
        if int(os.environ.get("WORLD_SIZE", "1")) != 1:
            sys.exit("bench.py --node: one process per node (not under torchrun)")
        t_node = time.time()

        def progress_node(msg):
            print(f"[bench {time.time() - t_node:7.1f} s] {msg}", file=sys.stderr, flush=True)
        node_main(args, progress_node)
        return
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(relaunch_under_torchrun(args, sys.argv[1:]))
    if int(os.environ.get("WORLD_SIZE", "1")) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={os.environ.get('WORLD_SIZE')} but --gpus {args.gpus}")
    # progress lines on stderr (stdout carries the one JSON line): phases
    # here, keygen waves from the C++ driver
    os.environ.setdefault("MPCX_PROGRESS", "1")
    t_start = time.time()

    # a native crash prints every thread's Python stack, and the module map
    # (rewritten at every phase, so it lists each library loaded so far) lets
    # a native stack's addresses be resolved afterwards
    import faulthandler
    faulthandler.enable()
    maps_path = os.path.abspath(args.detail) + f".maps.rank{os.environ.get('RANK', '0')}.txt"

    def progress(msg):
        print(f"[bench {time.time() - t_start:7.1f} s] {msg}", file=sys.stderr, flush=True)
        try:
            os.makedirs(os.path.dirname(maps_path), exist_ok=True)
            with open("/proc/self/maps") as fi, open(maps_path, "w") as fo:
                fo.write(fi.read())
        except OSError:
            pass

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = gpu_index()
    # clock / power / temperature of this rank's GPU over the timed region
    # (rank 0; a separate process, started before this one initialises the GPU)
    smi = SmiSampler(local) if rank == 0 and not args.no_smi else None
    # The signing CPU baseline forks worker processes: run it before this
    # process touches the GPU.
    info = host_info()
    if args.cpu_threads:
        info["usable_threads"] = args.cpu_threads
    sign_cpu = sign3_cpu = None
    if args.wallets > 0 and rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("CPU baseline: signing")
        sign_cpu = cpu_baseline_signing(args.cpu_sign_seconds, info, args.signers)
        if args.signers != 3:
            sign3_cpu = cpu_baseline_signing(args.cpu_sign_seconds, info, 3)
    keygen_cpu = None
    if args.keygen_sessions > 0 and rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("CPU baseline: keygen proofs")
        keygen_cpu = cpu_baseline_keygen(16.0, info, args.parties)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # gloo prints its connection messages to stdout from C++: keep stdout
        # for the one JSON result line by pointing fd 1 at stderr meanwhile
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            sys.stdout.flush()
            os.dup2(saved, 1)
            os.close(saved)
    torch.cuda.set_device(local)

    from mpcium_amd import build, mpcx
    if rank == 0 and not os.path.exists(os.path.join(ROOT, "mpcium_amd", "libmpcx.so")):
        build.build()
    if world > 1:
        dist.barrier()
    mpcx.init(local)
    for kv in args.opt:
        k, v = kv.split("=")
        mpcx.set_option(k, int(v))

    N = load_key()
    N2 = N * N if args.modbits == 4096 else N  # the modulus
    mod = mpcx.Modulus(N2)
    words = mod.words  # 128 for N^2; 64 for a 2048-bit N (operands below the lane-pair geometry's R)
    count = args.count
    bases = synth_bases(N2, count, 0x6D706332 + rank, words)
    exp = mpcx.int_to_words(N, mpcx.nwords(N))
    dev = torch.device("cuda", local)
    d_bases = torch.from_numpy(bases.view(np.int32)).to(dev)
    d_exp = torch.from_numpy(exp.view(np.int32)).to(dev)
    d_out = torch.zeros((count, words), dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev)
    L = mpcx.lib()

    def step():
        rc = L.mpcx_modexp_batch_device(mod.handle, count, d_bases.data_ptr(), words, d_exp.data_ptr(),
                                        len(exp), 1, N.bit_length(), d_out.data_ptr(), words,
                                        stream.cuda_stream)
        if rc != 0:
            raise mpcx.MpcxError(rc, L.mpcx_last_error().decode())

    progress("config 2: warm-up")
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    progress("config 2: timed steps")

    # one HIP event pair per timed step, on the launch stream (the library's
    # kernels run on `stream`, so the events bracket exactly one launch each)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    w0 = time.time()
    ev0.record(stream)
    for a, b in evs:
        a.record(stream)
        step()
        b.record(stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    w1 = time.time()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kernel_ms = ev0.elapsed_time(ev1) / args.steps  # one launch per step on `stream`
    step_ms = [a.elapsed_time(b) for a, b in evs]
    smi_window = smi.window(w0, w1) if smi else None

    # untimed correctness sample of the last step's outputs (after the timed
    # region so that --warmup 0 still checks real results)
    if args.verify and args.steps + args.warmup > 0:
        out = d_out.cpu().numpy().view(np.uint32)
        idx = np.linspace(0, count - 1, args.verify).astype(int)
        xs = mpcx.words_to_ints(bases[idx])
        zs = mpcx.words_to_ints(out[idx])
        bad = [int(i) for i, x, z in zip(idx, xs, zs) if pow(x, N, N2) != z]
        if bad:
            raise SystemExit(f"rank {rank}: GPU results differ from pow() at operands {bad[:5]}")

    # whole-batch digest of rank 0's default batch against the C restatement
    # (tests/golden/batch_digest.json, untimed)
    digest = None
    gd_path = os.path.join(ROOT, "tests", "golden", "batch_digest.json")
    if rank == 0 and args.modbits == 4096 and args.steps + args.warmup > 0 and os.path.exists(gd_path):
        gd = json.load(open(gd_path))
        if gd["count"] == count and gd["words"] == words:
            import hashlib
            got = hashlib.sha256(d_out.cpu().numpy().astype("<u4").tobytes()).hexdigest()
            digest = {"sha256": got, "expected": gd["sha256"], "match": got == gd["sha256"],
                      "scope": f"all {count} outputs of rank 0 vs oracle/gomodexp.c (tests/golden/batch_digest.json)"}
            if not digest["match"]:
                raise SystemExit(f"rank 0: batch digest {got} != C restatement {gd['sha256']}")

    def per_operand(E: int) -> dict:
        """Config-2 secondary shape: the same 65,536 bases with per-operand
        uniform E-bit exponents (Go's 4-bit fixed window per operand; no
        shared sliding-window schedule), one launch, HIP events."""
        rng = np.random.default_rng(0x70657230 + E)
        ew = (E + 31) // 32
        ex = rng.integers(0, 1 << 32, size=(count, ew), dtype=np.uint64).astype(np.uint32)
        tb = (E - 1) % 32
        ex[:, ew - 1] &= np.uint32((1 << (tb + 1)) - 1 if tb < 31 else 0xFFFFFFFF)
        ex[:, ew - 1] |= np.uint32(1 << tb)
        d_e = torch.from_numpy(ex.view(np.int32)).to(dev)
        d_o = torch.zeros((count, words), dtype=torch.int32, device=dev)

        def st():
            rc = L.mpcx_modexp_batch_device(mod.handle, count, d_bases.data_ptr(), words, d_e.data_ptr(), ew, 0, E,
                                            d_o.data_ptr(), words, stream.cuda_stream)
            if rc != 0:
                raise mpcx.MpcxError(rc, L.mpcx_last_error().decode())
        st()
        torch.cuda.synchronize()
        reps = 3
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for _ in range(reps):
            st()
        e1.record(stream)
        torch.cuda.synchronize()
        kms = e0.elapsed_time(e1) / reps
        out = d_o.cpu().numpy().view(np.uint32)
        idx = np.linspace(0, count - 1, 8).astype(int)
        xs, zs = mpcx.words_to_ints(bases[idx]), mpcx.words_to_ints(out[idx])
        es = mpcx.words_to_ints(ex[idx])
        if any(pow(x, e, N2) != z for x, e, z in zip(xs, es, zs)):
            raise SystemExit(f"per-operand {E}-bit exponents: GPU results differ from pow()")
        Wp = alg_macs(N2.bit_length(), E)
        ach = Wp * count / (kms * 1e-3)
        return {"exp_bits": E, "value": count / (kms * 1e-3), "unit": "modexp/s", "kernel_ms": kms,
                "roofline": {"bound": "valu", "achieved": ach / 1e12, "peak": PEAK_INT32_NOMINAL / 1e12,
                             "unit": "TOP/s", "frac": ach / PEAK_INT32_NOMINAL, "alg_ops_per_modexp": Wp},
                "checked": "8 sampled operands vs pow()"}

    sub_lines = None
    if rank == 0 and args.extra_lines and args.modbits == 4096:
        progress("config 2: per-operand exponents")
        sub_lines = [per_operand(2048), per_operand(4096)]

    from mpcium_amd.shard import max_over_ranks
    elapsed, kernel_ms = max_over_ranks([elapsed, kernel_ms], world)

    total = count * world * args.steps
    value = total / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    W = alg_macs(N2.bit_length(), N.bit_length())
    achieved = W * count / (kernel_ms * 1e-3)  # per GPU, per launch
    result = {
        "metric": METRIC,
        "value": value,
        "unit": "modexp/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32",
        "data": "synthetic: bases from numpy default_rng(0x6d706332+rank) clamped below N^2; N = product of two "
                "seeded 1024-bit safe primes (tests/golden/paillier_key_2048.json)",
        "config": {"workload": ("config2: x^N mod N^2, 4096-bit modulus, shared 2048-bit exponent y=N"
                                if args.modbits == 4096 else
                                "x^N mod N, 2048-bit modulus, shared 2048-bit exponent (N / N~ class)"),
                   "operands_per_gpu": count, "modulus_bits": N2.bit_length(), "exp_bits": N.bit_length(),
                   "parallelism": f"shard{world} (independent operands, no collective)",
                   "kernel_geometry": {"L": mod.L, "P": mod.P, "K": mod.K, "G": mod.G}},
        "roofline": {"bound": "valu", "achieved": achieved / 1e12, "peak": PEAK_INT32_NOMINAL / 1e12,
                     "unit": "TOP/s", "frac": achieved / PEAK_INT32_NOMINAL, "traffic": None,
                     "peak_measured_mad": PEAK_MAD_MEASURED / 1e12,
                     "frac_of_measured_mad": achieved / PEAK_MAD_MEASURED,
                     "alg_ops_per_modexp": W, "kernel_ms": kernel_ms},
        "cpu_baseline": None,
    }
    mx_on = (args.modbits == 4096 and (mod.P, mod.K) == (4, 37) and mpcx.get_option("mx") == 1
             and count >= mpcx.get_option("mx_min"))
    result["roofline"].update(pmc_traffic(count, args.modbits, mod, mx_on))
    result["roofline"]["kernel"] = "k_modexp_mx" if mx_on else "k_modexp<4, 37, 16, 2>"
    if mx_on:
        result["roofline"]["executed_floor"] = mx_floor(count, N, kernel_ms)
    if step_ms:
        srt = sorted(step_ms)
        q = max(1, len(step_ms) // 4)
        result["step_kernel_ms"] = {
            "min": srt[0], "median": srt[len(srt) // 2], "max": srt[-1],
            "first_quarter_mean": sum(step_ms[:q]) / q, "last_quarter_mean": sum(step_ms[-q:]) / q,
            "per_step": [round(x, 3) for x in step_ms],
            "note": "HIP events around each timed step on the launch stream (k_expsched + k_modexp)"}
    if smi is not None:
        smi.stop()
        result["gpu_telemetry"] = smi_window
        if smi_window:
            smi_window["scope"] = "amdsmi GPU metrics sampled every ~0.1 s by a separate process during the timed steps"
            clk = (smi_window.get("current_gfxclk") or {}).get("mean")
            if clk:  # the same work against the INT32 peak at the clock the GPU actually ran
                peak_clk = 256 * 64 * clk * 1e6
                result["roofline"]["gfxclk_mhz_measured"] = clk
                result["roofline"]["frac_at_measured_clock"] = achieved / peak_clk
    if result["roofline"].get("executed_floor"):
        two_pipe_roofline(result["roofline"])
    if digest:
        result["batch_digest"] = digest
    if sub_lines:
        result["config2_per_operand_exponents"] = sub_lines
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("CPU baseline: config 2")
        result["cpu_baseline"] = cpu_baseline(N, args.cpu_seconds, info)
    if args.wallets > 0:
        progress(f"config 4: signing, {args.signers} signers")
        result["signing"] = signing_line(args, world, rank, args.signers)
        result["signing"]["cpu_baseline"] = sign_cpu
        # mpcium signs with every ready peer (/root/reference/pkg/mpc/node.go:148)
        if args.signers != 3 and not args.no_sign3:
            progress("config 4: signing, 3 signers")
            result["signing_3_signers"] = signing_line(args, world, rank, 3)
            result["signing_3_signers"]["cpu_baseline"] = sign3_cpu
    if args.extra_lines:
        cpu = rank == 0 and world == 1 and not args.no_cpu_baseline
        progress("config 1 and 3: Paillier batch, safe primes")
        result["paillier_batch"] = paillier_line(N, 1024, 20, cpu, info, world, rank, args.paillier_inflight)
        result["safe_prime"] = safeprime_line(args.safe_primes, 0x5AFE, cpu, info, world, rank)
    if args.keygen_sessions > 0:
        progress(f"config 5: keygen/reshare proofs, {args.keygen_sessions} sessions per GPU")
        result["keygen"] = keygen_line(args, world, rank)
        result["keygen"]["cpu_baseline"] = keygen_cpu
    progress("done")
    result["host_copies"] = {"libmpcx": mpcx.copy_stats(), "maps": os.path.relpath(maps_path, ROOT),
                             "note": "direct: DMA from/to mpcx_host_alloc blocks; bounced: copied by libmpcx through "
                                     "its lanes' pinned buffers (no pageable pointer reaches hipMemcpyAsync)"}
    try:
        from mpcium_amd import host as mhost
        if mhost._lib is not None:
            result["host_copies"]["engine_pinned_pool"] = mhost.pinned_pool_stats()
    except Exception as ex:  # noqa: BLE001 -- diagnostics only
        result["host_copies"]["engine_pinned_pool"] = f"unavailable: {ex}"
    if rank == 0:
        detail = os.path.abspath(args.detail)
        os.makedirs(os.path.dirname(detail), exist_ok=True)
        with open(detail, "w") as f:
            json.dump(result, f, indent=1)
        print(json.dumps(compact_line(result, os.path.relpath(detail, ROOT))), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
