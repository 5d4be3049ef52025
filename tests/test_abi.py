"""CPU tests of the drop-in boundary: libmpcx.so builds for gfx950, exports
every entry point include/mpcx.h declares, and fails loudly (no CPU
fallback) when no GPU is present."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


@pytest.fixture(scope="module")
def libs():
    from mpcium_amd import build
    return build.build()


def header_functions(path):
    txt = open(path).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\bint\s+(mpcx_\w+)\s*\(", txt)) | set(re.findall(r"\bchar\s*\*\s*(mpcx_\w+)\s*\(", txt)))


def test_header_symbols_exported(libs):
    names = header_functions(os.path.join(ROOT, "include", "mpcx.h"))
    assert "mpcx_modexp_batch" in names and "mpcx_fermat2_batch" in names and "mpcx_last_error" in names
    lib = ctypes.CDLL(libs["libmpcx"])
    for n in names:
        assert hasattr(lib, n), n


def test_python_binding_covers_header(libs):
    from mpcium_amd import mpcx
    names = set(header_functions(os.path.join(ROOT, "include", "mpcx.h")))
    bound = {n for n, _, _ in mpcx.SIGNATURES}
    assert names == bound


def test_kernel_code_object_is_gfx950(libs):
    data = open(libs["libmpcx"], "rb").read()
    assert b"gfx950" in data


def test_fails_loudly_without_gpu(libs):
    from mpcium_amd import mpcx
    if mpcx.device_count() > 0:
        pytest.skip("GPU present")
    with pytest.raises(mpcx.MpcxError) as ei:
        mpcx.init(0)
    assert ei.value.code == mpcx.MPCX_ENODEV
    with pytest.raises(mpcx.MpcxError):
        mpcx.Modulus(65537)
    with pytest.raises(mpcx.MpcxError):
        mpcx.fermat2_batch([101])


def test_missing_library_raises(monkeypatch, tmp_path):
    from mpcium_amd import mpcx
    monkeypatch.setattr(mpcx, "_LIB_PATH", str(tmp_path / "nope.so"))
    monkeypatch.setattr(mpcx, "_lib", None)
    with pytest.raises(mpcx.MpcxError):
        mpcx.lib()


def test_device_partition_plan(libs):
    """The host-buffer batch split across a node's GPUs (mpcx_partition, the
    plan run_sliced executes): contiguous, disjoint, covering, balanced, and
    one range when the slices would be smaller than min_slice."""
    from mpcium_amd import mpcx
    for count in (0, 1, 4095, 8191, 8192, 65536, 65537, 100003):
        for ndev in (1, 2, 3, 4, 8):
            for mn in (0, 1, 4096):
                plan = mpcx.partition(count, ndev, mn)
                assert 1 <= len(plan) <= ndev
                assert plan[0][0] == 0 and sum(n for _, n in plan) == count
                for (f0, n0), (f1, _) in zip(plan, plan[1:]):
                    assert f0 + n0 == f1
                if mn == 0 or count < 2 * mn:
                    assert len(plan) == 1
                else:
                    assert len(plan) == min(ndev, count // mn)
                    assert max(n for _, n in plan) - min(n for _, n in plan) <= len(plan)
    with pytest.raises(mpcx.MpcxError):
        mpcx.partition(10, 0, 1)


def test_no_undefined_library_symbols():
    """Every mpcx_* symbol libmpcx.so references is defined in it (a launcher
    declared extern "C" but defined with C++ linkage fails only at load time)."""
    import subprocess
    so = os.path.join(ROOT, "mpcium_amd", "libmpcx.so")
    out = subprocess.run(["nm", "-D", "--undefined-only", so], capture_output=True, text=True, check=True).stdout
    assert [l for l in out.splitlines() if " mpcx" in l] == []
