"""mpcium_amd -- MI355X-native batched modular exponentiation for mpcium's
tss-lib hot path (Paillier mod N^2, MtA proofs, safe-prime search).

The product is libmpcx.so (C-ABI, include/mpcx.h) plus libmpcx_host.so (C++
mirror of tss-lib's ModInt.Exp / crypto/paillier / safe-prime interfaces).
This Python package only loads them through ctypes; it never computes a
modexp itself, and raises if the native libraries are missing.
"""
from .mpcx import (  # noqa: F401
    MpcxError,
    Modulus,
    device_count,
    exp_batch,
    fermat2_batch,
    mr_batch,
    init,
    lib,
    shutdown,
)

__version__ = "0.1.0"
