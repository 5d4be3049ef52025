"""GPU parity of the batched secp256k1 combination kernel (libmpcx
mpcx_ec_combine_batch: out = a G + b P + c Q, one thread per item) against the
oracle's affine restatement (oracle/tss_ref.py ec_add / ec_mul), bit-exact:
random combinations of every shape GG18 signing issues (a G; b P; a G + b P;
a G + b P + c Q), and the edge cases -- zero scalars, the point at infinity as
input and as result (b P + c (-P), a G - a G), equal and opposite points inside
the additions, scalars >= n, the generator as P."""
import pytest

from oracle import tss_ref as T

pytestmark = pytest.mark.gpu

Q = T.SECP_N


@pytest.fixture(scope="module")
def mx(gpu):
    from mpcium_amd import mpcx
    mpcx.init(0)
    return mpcx


def ref(a, b, c, P, Qp):
    r = T.scalar_base_mult(a)
    if P is not None:
        r = T.ec_add(r, T.ec_mul(b, P))
    if Qp is not None:
        r = T.ec_add(r, T.ec_mul(c, Qp))
    return r


def neg(P):
    return (P[0], T.SECP_P - P[1])


def test_random_combinations(mx):
    rd = T.Reader(0xEC01)
    rnd = lambda: T.get_random_positive_int(rd, Q)  # noqa: E731
    items = []
    for k in range(300):
        P = T.scalar_base_mult(rnd())
        Qp = T.scalar_base_mult(rnd())
        shape = k % 4
        if shape == 0:
            items.append((rnd(), 0, 0, None, None))
        elif shape == 1:
            items.append((0, rnd(), 0, P, None))
        elif shape == 2:
            items.append((rnd(), rnd(), 0, P, None))
        else:
            items.append((rnd(), rnd(), rnd(), P, Qp))
    got = mx.ec_combine_batch(items)
    assert got == [ref(*it) for it in items]


def test_edge_cases(mx):
    G = T.SECP_G
    P = T.scalar_base_mult(0x1234567890ABCDEF)
    k = 0xDEADBEEF12345678
    items = [
        (0, 0, 0, None, None),            # nothing: infinity
        (1, 0, 0, None, None),            # G
        (Q - 1, 0, 0, None, None),        # -G
        (Q, 0, 0, None, None),            # n G = infinity
        (Q + 5, 0, 0, None, None),        # scalar >= n
        (2 ** 256 - 1, 0, 0, None, None),
        (0, 1, 0, P, None),               # P
        (0, Q, 0, P, None),               # n P = infinity
        (0, 3, 3, P, neg(P)),             # 3P - 3P = infinity
        (0, k, k, P, P),                  # doubling inside the Shamir additions
        (k, k, 0, G, None),               # k G + k G: doubling in the mixed addition
        (k, Q - k, 0, G, None),           # k G - k G = infinity
        (5, 0, 7, None, P),               # only Q
        (5, 9, 7, P, None),               # Q infinite with c != 0
        (0, 2 ** 255 + 3, 1, G, G),
        (2 ** 256 + 7, 0, 0, None, None),  # scalars >= 2^256 and negative: mod n
        (-5, 2 ** 300 + 1, -(2 ** 260), P, G),
    ]
    got = mx.ec_combine_batch(items)
    assert got == [ref(*it) for it in items]


def test_ragged_batch_sizes(mx):
    rd = T.Reader(0xEC02)
    for n in (1, 63, 64, 65, 129):
        items = [(T.get_random_positive_int(rd, Q), T.get_random_positive_int(rd, Q), 0,
                  T.scalar_base_mult(i + 2), None) for i in range(n)]
        assert mx.ec_combine_batch(items) == [ref(*it) for it in items]
