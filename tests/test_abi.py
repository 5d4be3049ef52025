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
