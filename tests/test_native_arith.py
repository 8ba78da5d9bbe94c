"""The kernel arithmetic headers (hbbft_amd/csrc/*.h) compiled for the HOST and checked
against the Python oracle (oracle/bls12_381.py): codec, scalar multiplication, Miller loop
value, final exponentiation (HHT chain = cube of the pairing), pairing-equality checks and
the endomorphism subgroup tests.  Runs without a GPU."""
import ctypes
import os
import random
import subprocess

import pytest

from oracle import bls12_381 as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "libhbtc_hosttest.so")


@pytest.fixture(scope="module")
def ht():
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(
            os.path.getmtime(os.path.join(ROOT, "hbbft_amd", "csrc", f))
            for f in ("field.h", "curve.h", "pairing.h", "bls_constants.h")):
        subprocess.check_call(["make", "-s", "-C", ROOT, "hosttest"])
    return ctypes.CDLL(LIB)


def buf(n):
    return ctypes.create_string_buffer(n)


def tower(e):
    out = []
    for k in (0, 2, 4, 1, 3, 5):
        out += [(e[k] + e[k + 6]) % B.P, e[k + 6]]
    return out


def read12(raw):
    return [int.from_bytes(raw[48 * i:48 * i + 48], "big") for i in range(12)]


def test_generators_decode(ht):
    ox, oy = buf(48), buf(48)
    assert ht.ht_g1_decompress(B.g1_compress(B.G1_GEN), ox, oy) == 0
    assert (int.from_bytes(ox.raw, "big"), int.from_bytes(oy.raw, "big")) == B.G1_GEN
    o = buf(192)
    assert ht.ht_g2_decompress(B.g2_compress(B.G2_GEN), o) == 0
    assert o.raw == B.g2_uncompress_bytes(B.G2_GEN)


def test_codec_and_mul_roundtrip(ht):
    rng = random.Random(1)
    g1, g2 = B.g1_compress(B.G1_GEN), B.g2_compress(B.G2_GEN)
    for _ in range(4):
        k = rng.randrange(B.R)
        P, Q = B.g1_mul(B.G1_GEN, k), B.g2_mul(B.G2_GEN, k)
        o1, o2 = buf(48), buf(96)
        assert ht.ht_g1_roundtrip(B.g1_compress(P), o1) == 0 and o1.raw == B.g1_compress(P)
        assert ht.ht_g2_roundtrip(B.g2_compress(Q), o2) == 0 and o2.raw == B.g2_compress(Q)
        ks = k.to_bytes(32, "little")
        assert ht.ht_g1_mul(g1, ks, o1) == 0 and o1.raw == B.g1_compress(P)
        assert ht.ht_g2_mul(g2, ks, o2) == 0 and o2.raw == B.g2_compress(Q)


def test_glv_split_scalar_of_rlc_items(ht):
    """r_i d_i = [a] d + [b] phi(d) equals [a + b mu] d with mu = -x^2 mod r (the eigenvalue of
    phi(x, y) = (beta x, y) on G1): the RLC scalars are a + b mu for the two 32-bit halves of a
    ChaCha20 word, and distinct (a, b) give distinct residues mod r."""
    rng = random.Random(5)
    mu = (-(B.X * B.X)) % B.R
    cases = [(0, 0), (1, 0), (0, 1), (0xffffffff, 0xffffffff), (1, 0xffffffff)]
    cases += [(rng.getrandbits(32), rng.getrandbits(32)) for _ in range(4)]
    ht.ht_g1_mul_glv32.argtypes = [ctypes.c_char_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_char_p]
    for a, b in cases:
        P = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
        o = buf(48)
        assert ht.ht_g1_mul_glv32(B.g1_compress(P), a, b, o) == 0
        assert o.raw == B.g1_compress(B.g1_mul(P, (a + b * mu) % B.R)), (a, b)


@pytest.mark.parametrize("nbits", [16, 32])
def test_xadic_scalar_of_rlc_items(ht, nbits):
    """The x-adic RLC scalar (curve.h xadic_mul_uniform, rlc_common.h rlc_digits): the item passes
    compute [d0] P + [d1] [x]P + [d2] m(P) + [d3] m([x]P) with m the endomorphism of eigenvalue
    mu = -x^2 (G1: phi, G2: -psi^2) and [x]P = -[|x|]P from the G1 subgroup test / psi(P) on G2;
    it must equal [d0 + d1 x + d2 mu + d3 mu x] P, for 16- and 32-bit digits (64- / 128-bit RLC)."""
    rng = random.Random(nbits)
    mu = (-(B.X * B.X)) % B.R
    top = (1 << nbits) - 1
    cases = [(0, 0, 0, 0), (1, 0, 0, 0), (0, 1, 0, 0), (0, 0, 1, 0), (0, 0, 0, 1), (top,) * 4,
             (1, top, 0, top)]
    cases += [tuple(rng.getrandbits(nbits) for _ in range(4)) for _ in range(4)]
    ht.ht_g1_mul_xadic.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    ht.ht_g2_mul_xadic.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    ht.ht_g1_mul_xadic8.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    ht.ht_g2_mul_xadic8.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    ht.ht_g2_mul_xadic_lds.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    ht.ht_g1_mul_xadic8_lds.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    ht.ht_g2_mul_xadic8_lds.argtypes = [ctypes.c_char_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p]
    cases += [(2, 0, 0, 0), (0, top, top, top), (top - 1, 1, 1, 1), (2, 1, 0, 0)]
    for d in cases:
        r = (d[0] + d[1] * B.X + d[2] * mu + d[3] * mu * B.X) % B.R
        arr = (ctypes.c_uint32 * 4)(*d)
        P = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
        o = buf(48)
        assert ht.ht_g1_mul_xadic(B.g1_compress(P), ctypes.cast(arr, ctypes.c_void_p), nbits, o) == 0
        assert o.raw == B.g1_compress(B.g1_mul(P, r)), ("g1", d)
        Q = B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))
        o2 = buf(96)
        assert ht.ht_g2_mul_xadic(B.g2_compress(Q), ctypes.cast(arr, ctypes.c_void_p), nbits, o2) == 0
        assert o2.raw == B.g2_compress(B.g2_mul(Q, r)), ("g2", d)
        # k_sig_items' form: the same loop over the table in an LDS-layout buffer
        assert ht.ht_g2_mul_xadic_lds(B.g2_compress(Q), ctypes.cast(arr, ctypes.c_void_p), nbits, o2) == 0
        assert o2.raw == B.g2_compress(B.g2_mul(Q, r)), ("g2 lds", d)
        # the sign-aligned 8-entry form (curve.h xadic_mul_sac8), even d0 included
        assert ht.ht_g1_mul_xadic8(B.g1_compress(P), ctypes.cast(arr, ctypes.c_void_p), nbits, o) == 0
        assert o.raw == B.g1_compress(B.g1_mul(P, r)), ("g1 sac8", d)
        assert ht.ht_g2_mul_xadic8(B.g2_compress(Q), ctypes.cast(arr, ctypes.c_void_p), nbits, o2) == 0
        assert o2.raw == B.g2_compress(B.g2_mul(Q, r)), ("g2 sac8", d)
        # k_rlc_items' form: three entries in an LDS-layout buffer, the co-Z chain build
        assert ht.ht_g1_mul_xadic8_lds(B.g1_compress(P), ctypes.cast(arr, ctypes.c_void_p), nbits, o) == 0
        assert o.raw == B.g1_compress(B.g1_mul(P, r)), ("g1 sac8 lds", d)
        assert ht.ht_g2_mul_xadic8_lds(B.g2_compress(Q), ctypes.cast(arr, ctypes.c_void_p), nbits, o2) == 0
        assert o2.raw == B.g2_compress(B.g2_mul(Q, r)), ("g2 sac8 lds", d)


def test_sac2_two_digit_form(ht):
    """The small combines' scalar multiplication (curve.h sac2_mul): [d0] P + [d1] [u] P, u = |x|,
    for 64-bit digits (base-u digits of Lagrange coefficients, so the edge digits are covered too:
    zero, even / odd d0, all-ones, u - 1) on G1 and G2."""
    rng = random.Random(77)
    u = abs(B.X)
    top = (1 << 64) - 1
    cases = [(0, 0), (1, 0), (0, 1), (2, 0), (2, 1), (top, top), (u - 1, u - 1), (u - 2, 1), (0, u - 1)]
    cases += [(rng.getrandbits(64), rng.getrandbits(64)) for _ in range(6)]
    ht.ht_g1_mul_sac2.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p]
    ht.ht_g2_mul_sac2.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_char_p]
    for d0, d1 in cases:
        k = (d0 + d1 * u) % B.R
        P = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
        o = buf(48)
        assert ht.ht_g1_mul_sac2(B.g1_compress(P), d0, d1, o) == 0
        assert o.raw == B.g1_compress(B.g1_mul(P, k)), ("g1", d0, d1)
        Q = B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))
        o2 = buf(96)
        assert ht.ht_g2_mul_sac2(B.g2_compress(Q), d0, d1, o2) == 0
        assert o2.raw == B.g2_compress(B.g2_mul(Q, k)), ("g2", d0, d1)


def test_xadic_digit_box_is_injective():
    """2^(4 nbits) distinct digit vectors give distinct residues: d0 + d1 x - d2 x^2 - d3 x^3 with
    |d_j| < 2^33 < |x| is below r in absolute value and zero only for zero digits (digit by digit
    mod x); checked here on the extreme differences."""
    X = B.X
    assert abs(X) > 1 << 33
    worst = (1 << 33) * (1 + abs(X) + X * X + abs(X) ** 3)
    assert worst < B.R
    for d in [(1, 0, 0, 0), (0, 1, 0, 0), (-(1 << 32), 1 << 32, -(1 << 32), 1 << 32)]:
        v = d[0] + d[1] * X - d[2] * X * X - d[3] * X ** 3
        assert v != 0 and v % B.R != 0


def test_miller_loop_value_matches_oracle(ht):
    o = buf(576)
    assert ht.ht_miller(B.g1_compress(B.G1_GEN), B.g2_compress(B.G2_GEN), o) == 0
    assert read12(o.raw) == tower(B.miller_loop(B.G1_GEN, B.G2_GEN))


def test_final_exponentiation_is_cube_of_pairing(ht):
    o = buf(576)
    assert ht.ht_pairing(B.g1_compress(B.G1_GEN), B.g2_compress(B.G2_GEN), o) == 0
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert read12(o.raw) == tower(B.f12_mul(B.f12_mul(e, e), e))


def test_pairing_equality_checks(ht):
    rng = random.Random(2)
    c, d = B.g1_compress, B.g2_compress
    a, b = rng.randrange(B.R), rng.randrange(B.R)
    P1, Q1 = B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)
    P2, Q2 = B.g1_mul(B.G1_GEN, a * b % B.R), B.G2_GEN
    for fn in (ht.ht_pairing_eq, ht.ht_pairing_eq_var):
        assert fn(c(P1), d(Q1), c(P2), d(Q2)) == 1
        assert fn(c(P1), d(Q1), c(B.g1_neg(P2)), d(Q2)) == 0
        assert fn(c(P1), d(Q1), c(P2), d(B.g2_neg(Q2))) == 0
        # identities: e(O, Q) = 1
        assert fn(c(None), d(Q1), c(P2), d(None)) == 1
        assert fn(c(None), d(Q1), c(P2), d(Q2)) == 0


def _rand_curve(rng, g):
    while True:
        if g == 1:
            p = B.g1_point_from_x(rng.randrange(B.P), False)
        else:
            p = B.g2_point_from_x((rng.randrange(B.P), rng.randrange(B.P)), False)
        if p:
            return p


def _small_component(rng, g, prime, h):
    """A point of order `prime` in E(Fq) (g=1) / E'(Fq2) (g=2).  The prime-power part of
    the group can be non-cyclic, so strip the full prime power from the multiplier."""
    e = 0
    n = h
    while n % prime == 0:
        n //= prime
        e += 1
    for _ in range(64):
        p = _rand_curve(rng, g)
        t = (B.g1_mul if g == 1 else B.g2_mul)(p, n * B.R)  # now order | prime^e
        for _ in range(e):
            nxt = (B.g1_mul if g == 1 else B.g2_mul)(t, prime)
            if nxt is None:
                break
            t = nxt
        if t is not None:
            return t
    raise AssertionError("no point of order %d found" % prime)


def _xy(g, pt):
    if g == 1:
        return pt[0].to_bytes(48, "big") + pt[1].to_bytes(48, "big")
    return B.g2_uncompress_bytes(pt)


def test_g1_subgroup_test_matches_r_torsion(ht):
    rng = random.Random(3)
    for _ in range(6):
        p = _rand_curve(rng, 1)
        assert ht.ht_g1_subgroup_xy(_xy(1, p)) == int(B.g1_in_subgroup(p))
        assert ht.ht_g1_subgroup_xy(_xy(1, B.g1_mul(p, B.H1))) == 1
    base = B.g1_mul(B.G1_GEN, rng.randrange(B.R))
    for prime in (3, 11, 10177, 859267, 52437899):  # h1 = 3 * 11^2 * 10177^2 * 859267^2 * 52437899^2
        t = _small_component(rng, 1, prime, B.H1)
        assert ht.ht_g1_subgroup_xy(_xy(1, t)) == 0
        assert ht.ht_g1_subgroup_xy(_xy(1, B.g1_add(base, t))) == 0


def test_g2_subgroup_test_matches_r_torsion(ht):
    rng = random.Random(4)
    for _ in range(3):
        p = _rand_curve(rng, 2)
        assert ht.ht_g2_subgroup_xy(_xy(2, p)) == int(B.g2_in_subgroup(p))
        assert ht.ht_g2_subgroup_xy(_xy(2, B.g2_mul(p, B.H2))) == 1
    base = B.g2_mul(B.G2_GEN, rng.randrange(B.R))
    for prime in (13, 23):
        t = _small_component(rng, 2, prime, B.H2)
        assert ht.ht_g2_subgroup_xy(_xy(2, t)) == 0
        assert ht.ht_g2_subgroup_xy(_xy(2, B.g2_add(base, t))) == 0
