import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU; runs through libmpcx.so")


def load_golden(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


def H(s):
    if s is None:
        return None
    return -int(s[1:], 16) if s.startswith("-") else int(s, 16)


@pytest.fixture(scope="session")
def golden_modexp():
    return load_golden("modexp_vectors.json")["vectors"]


@pytest.fixture(scope="session")
def paillier_key():
    k = load_golden("paillier_key_2048.json")
    return {kk: (int(v, 16) if isinstance(v, str) and kk in ("P", "Q", "N", "LambdaN", "PhiN") else v) for kk, v in k.items()}


@pytest.fixture(scope="session")
def gpu():
    """Initialise libmpcx on cuda:0 (GPU tests only). Fails loudly without it."""
    from mpcium_amd import build, mpcx
    build.build()
    mpcx.init(0)
    return mpcx
