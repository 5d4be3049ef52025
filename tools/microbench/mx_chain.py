"""Check and time montmul_mx (mpcx_mx.hpp) against montmul<4, 37> on squaring chains.

    hipcc --offload-arch=gfx950 -O3 -shared -fPIC -o tools/microbench/mx_chain.so tools/microbench/mx_chain.hip
    python tools/microbench/mx_chain.py [count] [squarings] > result.json

1. the 16x16x64 i8 MFMA lane map this kernel relies on: C[4h + r][n] (lane n + 16h,
   register r) = sum over (h', e) of A-lane (row + 16h') byte e x B-lane (col + 16h')
   byte e -- A and B share the lane's k order, whatever it is;
2. the Toeplitz fragment tables of m'' = -m^-1 mod R and m (R = 2^4144), built here
   the way the C-ABI builds them;
3. both chains on the same operands: each result mod m must equal
   x^(2^S) R^-(2^S - 1) mod m (both kernels are Montgomery squarings in one domain),
   and the kernel times.
"""
import ctypes
import json
import os
import random
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", ".."))
from mpcium_amd import mpcx  # noqa: E402  (mpcx_mx_tables: host-only)

HERE = os.path.dirname(os.path.abspath(__file__))
L, DB = 148, 28
RBITS = L * DB
NJ1, NJ2 = 37, 41


def digits(v, n, bits):
    mask = (1 << bits) - 1
    return [(v >> (bits * i)) & mask for i in range(n)]


def from_digits(ds, bits):
    return sum(int(d) << (bits * i) for i, d in enumerate(ds))


def toeplitz(v7, nj):
    """[nj][64 lanes][16 bytes]: lane (i, h) byte e = v7[16 j + i - 16 h - e] (0 outside)."""
    out = bytearray(nj * 64 * 16)
    for j in range(nj):
        for lane in range(64):
            i, h = lane & 15, lane >> 4
            for e in range(16):
                idx = 16 * j + i - 16 * h - e
                if 0 <= idx < len(v7):
                    out[(j * 64 + lane) * 16 + e] = v7[idx]
    return bytes(out)


def model_step(a, b, m, m2):
    """One montmul_mx in plain integers, digit for digit as the kernel does it:
    returns (q's radix-2^28 digits e_d, U + m's digits u_d before the final carry pass)."""
    M28 = (1 << 28) - 1
    R = 1 << RBITS

    def i32(x):
        x &= 0xFFFFFFFF
        return x - (1 << 32) if x >= 1 << 31 else x

    def split(c, add):
        lo_sum = i32(c[0] + ((c[1] & 0x1FFFFF) << 7) + ((c[2] & 0x3FFF) << 14) + ((c[3] & 0x7F) << 21) + add)
        return lo_sum, (c[1] >> 21) + (c[2] >> 14) + (c[3] >> 7)

    T = a * b
    tl, th = digits(T % R, L, DB), digits(T >> RBITS, L, DB)
    t7, m27, m7 = digits(T % R, 592, 7), digits(m2, 592, 7), digits(m, 592, 7)
    c1 = [sum(t7[k] * m27[P - k] for k in range(P + 1)) for P in range(592)]
    e, hprev = [], 0
    for d in range(L):
        lo_sum, hi_sum = split(c1[4 * d:4 * d + 4], 1 << 27)
        e.append((lo_sum & M28) - (1 << 27) + hprev)
        hprev = hi_sum + (lo_sum >> 28)
    q7 = []
    for ed in e:
        x = ed & 0xFFFFFFFF
        for msk in (0xFFFFFF80, 0xFFFF8000, 0xFF800000):
            x = (x + (x & msk)) & 0xFFFFFFFF
        q7 += [((x >> (8 * i)) & 0xFF) - (256 if (x >> (8 * i)) & 0x80 else 0) for i in range(4)]
    c2 = [sum(q7[k] * m7[P - k] for k in range(max(0, P - 591), min(P, 591) + 1)) for P in range(1184)]
    lo_sum, hi_sum = split(c2[588:592], tl[147] + (1 << 27))
    cin = hi_sum + (lo_sum >> 28)
    md, u = digits(m, L, DB), []
    for d in range(L):
        lo_sum, hi_sum = split(c2[592 + 4 * d:596 + 4 * d], th[d] + md[d])
        hi = hi_sum + (lo_sum >> 28)
        u.append(i32(lo_sum + (hi_sum << 28)) + cin if d == L - 1 else (lo_sum & M28) + cin)
        cin = hi
    return e, u


def debug(lib, dev, rng):
    """S = 1 on 16 operands; R1 (q's bytes) and R0 (U + m) against model_step."""
    m = rng.getrandbits(4096) | (1 << 4095) | 1
    R = 1 << RBITS
    m2 = (-pow(m, -1, R)) % R
    imgd = torch.frombuffer(bytearray(mpcx.mx_tables(m, 148)), dtype=torch.uint8).to(dev)
    md = torch.tensor(digits(m, L, DB), dtype=torch.int64).to(torch.int32).to(dev)
    xs = [rng.randrange(m) for _ in range(16)]
    xd = torch.tensor([digits(v, L, DB) for v in xs], dtype=torch.int64).to(torch.int32).to(dev)
    out = torch.zeros_like(xd)
    dbg = torch.zeros(16 * L, dtype=torch.int32, device=dev)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    lib.mxb_chain_mx(vp(xd), vp(out), vp(imgd), vp(md), 1, 16, vp(dbg))
    torch.cuda.synchronize()
    rows = (dbg.cpu().to(torch.int64) & 0xFFFFFFFF).view(1, 16, L)
    rep = []
    for n in range(4):
        e, u = model_step(xs[n], xs[n], m, m2)
        qw = []
        for ed in e:
            x = ed & 0xFFFFFFFF
            for msk in (0xFFFFFF80, 0xFFFF8000, 0xFF800000):
                x = (x + (x & msk)) & 0xFFFFFFFF
            qw.append(x)
        got_q = qw  # q stays in registers (permlane transposes)
        got_u = [v - (1 << 32) if v >= 1 << 31 else v for v in rows[0, n].tolist()]
        bq = [d for d in range(L) if got_q[d] != qw[d]]
        bu = [d for d in range(L) if got_u[d] != u[d]]
        rep.append({"operand": n, "q_bad": len(bq), "q_first": bq[:6],
                    "q_pairs": [(qw[d], got_q[d]) for d in bq[:3]],
                    "u_bad": len(bu), "u_first": bu[:6], "u_pairs": [(u[d], got_u[d]) for d in bu[:3]]})
    return rep


def main():
    count = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    S = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    lib = ctypes.CDLL(os.path.join(HERE, os.environ.get("MX_CHAIN_SO", "mx_chain.so")))
    lib.mxb_chain_mx.restype = ctypes.c_float
    lib.mxb_chain_cios.restype = ctypes.c_float
    dev = torch.device("cuda:0")
    rng = random.Random(20261018)
    res = {}
    if len(sys.argv) > 3 and sys.argv[3] == "debug":
        print(json.dumps({"debug": debug(lib, dev, rng)}))
        return

    # 1. lane map
    a = torch.randint(-128, 128, (64, 16), dtype=torch.int8)
    b = torch.randint(-128, 128, (64, 16), dtype=torch.int8)
    ad, bd = a.to(dev), b.to(dev)
    cd = torch.zeros((64, 4), dtype=torch.int32, device=dev)
    assert lib.mxb_mfma_map(ctypes.c_void_p(ad.data_ptr()), ctypes.c_void_p(bd.data_ptr()),
                            ctypes.c_void_p(cd.data_ptr())) == 0
    c = cd.cpu()
    ai, bi = a.to(torch.int64), b.to(torch.int64)
    bad = 0
    for lane in range(64):
        n, h = lane & 15, lane >> 4
        for r in range(4):
            row = 4 * h + r
            want = sum(int((ai[row + 16 * hh] * bi[n + 16 * hh]).sum()) for hh in range(4))
            bad += int(c[lane, r]) != want
    res["mfma_map_mismatches"] = bad

    # 2. modulus and tables
    m = rng.getrandbits(4096) | (1 << 4095) | 1
    R = 1 << RBITS
    m2 = (-pow(m, -1, R)) % R
    imgd = torch.frombuffer(bytearray(mpcx.mx_tables(m, 148)), dtype=torch.uint8).to(dev)
    md = torch.tensor(digits(m, L, DB), dtype=torch.int64).to(torch.int32).to(dev)
    n0inv = (-pow(m, -1, 1 << DB)) % (1 << DB)

    # 3. chains (operands < m; a sample is checked against Python)
    xs = [rng.randrange(m) for _ in range(min(count, 64))]
    xs = (xs * ((count + len(xs) - 1) // len(xs)))[:count]
    xh = torch.tensor([digits(v, L, DB) for v in xs], dtype=torch.int64).to(torch.int32)
    xd = xh.to(dev)
    o_mx = torch.zeros_like(xd)
    o_ci = torch.zeros_like(xd)
    vp = lambda t: ctypes.c_void_p(t.data_ptr())
    # warm-up, then timed
    lib.mxb_chain_mx(vp(xd), vp(o_mx), vp(imgd), vp(md), 2, count, None)
    lib.mxb_chain_cios(vp(xd), vp(o_ci), vp(md), n0inv, 2, count)
    prof = None
    if os.environ.get("MX_PROF"):  # a build with -DMX_PROF: per-wave phase cycles after the rows
        prof = torch.zeros(16 * L + ((count + 15) // 16) * 8, dtype=torch.int32, device=dev)
    t_mx = lib.mxb_chain_mx(vp(xd), vp(o_mx), vp(imgd), vp(md), S, count, vp(prof) if prof is not None else None)
    t_ci = lib.mxb_chain_cios(vp(xd), vp(o_ci), vp(md), n0inv, S, count)
    torch.cuda.synchronize()
    omx, oci = o_mx.cpu().to(torch.int64) & 0xFFFFFFFF, o_ci.cpu().to(torch.int64) & 0xFFFFFFFF
    rinv = pow(R, -1, m)
    ok_mx = ok_ci = 0
    max_dig = 0
    over = 0
    for i in range(min(count, 64)):
        want = pow(xs[i], 1 << S, m) * pow(rinv, (1 << S) - 1, m) % m
        vmx = from_digits(omx[i].tolist(), DB)
        vci = from_digits(oci[i].tolist(), DB)
        ok_mx += vmx % m == want
        ok_ci += vci % m == want
        max_dig = max(max_dig, max(omx[i].tolist()))
        over += vmx >= 2 * m
    sq = count * S
    res.update({
        "count": count, "squarings": S, "checked": min(count, 64),
        "ok_mx": ok_mx, "ok_cios": ok_ci, "mx_max_digit": max_dig, "mx_values_ge_2m": over,
        "ms_mx": round(t_mx, 3), "ms_cios": round(t_ci, 3),
        "ns_per_squaring_mx": round(t_mx * 1e6 / sq, 4), "ns_per_squaring_cios": round(t_ci * 1e6 / sq, 4),
        "speedup": round(t_ci / t_mx, 3) if t_mx > 0 else None,
    })
    if prof is not None:
        pv = (prof.cpu().to(torch.int64) & 0xFFFFFFFF)[16 * L:].view(-1, 8)[:, :6].to(torch.float64) * 256 / S
        names = ["product", "fence_bfrag", "q_phase", "qm_emit", "fence", "carry_loop"]
        res["phase_cycles_per_squaring_mean_wave"] = {k: round(float(v), 1) for k, v in zip(names, pv.mean(0))}
        res["phase_cycles_total"] = round(float(pv.sum(1).mean()), 1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
