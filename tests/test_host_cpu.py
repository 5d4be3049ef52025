"""CPU tests of the C++ host mirror (libmpcx_host.so): pieces that need no
GPU -- the deterministic random stream and the tss-lib candidate layout --
against the oracle restatements, plus symbol coverage of mpcx_host.h."""
import ctypes
import os
import re

import pytest

from conftest import ROOT
from oracle import gomath as gm
from oracle import safeprime_ref as sp


@pytest.fixture(scope="module")
def hostlib():
    from mpcium_amd import build, host
    build.build()
    return host


def test_host_header_symbols(hostlib):
    txt = re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "mpcx_host.h")).read(), flags=re.S)
    names = set(re.findall(r"\b(mpcxh_\w+)\s*\(", txt))
    lib = ctypes.CDLL(hostlib._LIB_PATH)
    for n in names:
        assert hasattr(lib, n), n
    from mpcium_amd import mta, proofs
    assert names == ({n for n, _, _ in hostlib.SIGNATURES} | {n for n, _, _ in mta.SIGNATURES}
                     | {n for n, _, _ in proofs.SIGNATURES})


def test_drbg_matches_oracle(hostlib):
    for seed in (0, 1, 0x6D706331, 2 ** 64 - 1):
        assert hostlib.drbg_read(seed, 1000) == gm.CounterDRBG(seed).read(1000)
    # bulk reads (>= 64 KiB: counter blocks computed in parallel) give the same stream
    for n in (65536, 65536 + 17, 300001):
        assert hostlib.drbg_read(7, n) == gm.CounterDRBG(7).read(n)


def test_candidate_layout_matches_oracle(hostlib):
    rng = gm.CounterDRBG(99)
    for qbits in (63, 127, 255, 511, 1023, 5, 8, 9, 16):
        nb = (qbits + 7) // 8
        for _ in range(20):
            raw = rng.read(nb)
            assert hostlib.candidate_from_bytes(raw, qbits) == sp.candidate_from_bytes(raw, qbits), qbits


def test_host_fails_loudly_without_gpu(hostlib):
    from mpcium_amd import mpcx
    if mpcx.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(mpcx.MpcxError):
        hostlib.init(0)
    with pytest.raises(mpcx.MpcxError):
        hostlib.modint_exp(65537, [3], 5)
