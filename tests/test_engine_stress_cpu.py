"""CPU stress of the Engine's coalescers, pinned staging pool and comb-table
cache under AddressSanitizer + UBSan and ThreadSanitizer, against the CPU
mock of libmpcx (tools/mock_mpcx.cpp, tools/engine_stress.cpp): concurrent
comb and generic batches, comb tables rebuilt for longer exponents while
other threads still launch on the old ones, cache eviction under load, and
refused pinned allocations (the pageable fallback). Every output is checked
against the mock's result function."""
import os
import shutil
import subprocess

import pytest

from conftest import ROOT


@pytest.mark.parametrize("mode,iters", [("asan", 20), ("tsan", 20)])
def test_engine_stress_sanitized(mode, iters, tmp_path):
    if shutil.which("g++") is None:
        pytest.skip("no g++")
    env = dict(os.environ, TMPDIR=str(tmp_path), MOCK_PIN_FAIL="150")
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "engine_stress.sh"), mode, "10", str(iters)],
                       capture_output=True, text=True, env=env, timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "engine_stress: OK" in out
    assert "ERROR: AddressSanitizer" not in out and "WARNING: ThreadSanitizer" not in out
    assert "pageable buffer #1" in out  # the fallback is loud
