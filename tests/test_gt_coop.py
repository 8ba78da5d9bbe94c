"""The wavefront-cooperative GT arithmetic (hbbft_amd/csrc/gt6.h: one Fq12 over 6 lanes, one
Fq2 coefficient per lane) run on a host lane simulator (tests/native/gt_sim.cpp: one thread
per lane, meeting at every cross-lane exchange) against the serial tower arithmetic of
pairing.h / field.h, which tests/test_native_arith.py pins to the Python oracle.  This is the
same source the gfx950 check kernels (hbtc_check.hip) compile.  Runs without a GPU."""
import ctypes
import os
import random
import subprocess

import pytest

from oracle import bls12_381 as B

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "tests", "native", "libhbtc_hosttest.so")
HDRS = ("field.h", "curve.h", "pairing.h", "bls_constants.h", "gt6.h", "fq_fips.h")


@pytest.fixture(scope="module")
def ht():
    srcs = [os.path.join(ROOT, "hbbft_amd", "csrc", f) for f in HDRS]
    srcs.append(os.path.join(ROOT, "tests", "native", "gt_sim.cpp"))
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < max(os.path.getmtime(f) for f in srcs):
        subprocess.check_call(["make", "-s", "-C", ROOT, "hosttest"])
    return ctypes.CDLL(LIB)


def rand12(rng):
    return b"".join(rng.randrange(B.P).to_bytes(48, "big") for _ in range(12))


def op(lib, fn, code, a, b=None):
    out = ctypes.create_string_buffer(576)
    assert getattr(lib, fn)(code, a, b if b is not None else a, out) == 0
    return out.raw


def cyclotomic(ht, rng):
    """f^((p^6 - 1)(p^2 + 1)) of a random f, through the serial tower ops."""
    x = op(ht, "ht_tower_op", 8, rand12(rng))      # f^(p^6 - 1)
    return op(ht, "ht_tower_op", 0, op(ht, "ht_tower_op", 4, x), x)


@pytest.mark.parametrize("code,name", [(0, "mul"), (1, "sqr"), (3, "frob1"), (4, "frob2"),
                                       (5, "frob3"), (6, "conj")])
def test_gt_ops_match_tower(ht, code, name):
    rng = random.Random(100 + code)
    for _ in range(3):
        a, b = rand12(rng), rand12(rng)
        assert op(ht, "ht_gt_op", code, a, b) == op(ht, "ht_tower_op", code, a, b), name


def test_gt_cyclotomic_and_exp_by_x_match_tower(ht):
    rng = random.Random(7)
    c = cyclotomic(ht, rng)
    assert op(ht, "ht_gt_op", 2, c) == op(ht, "ht_tower_op", 2, c)
    assert op(ht, "ht_gt_op", 9, c) == op(ht, "ht_tower_op", 9, c)


def test_gt_easy_part_and_final_exp_match_tower(ht):
    rng = random.Random(8)
    f = rand12(rng)
    assert op(ht, "ht_gt_op", 8, f) == op(ht, "ht_tower_op", 8, f)
    assert op(ht, "ht_gt_op", 7, f) == op(ht, "ht_tower_op", 7, f)


def _check(ht, p1, q1, p2, q2, z1=1, z2=1):
    f, e = ctypes.create_string_buffer(576), ctypes.create_string_buffer(576)
    rc = ht.ht_gt_check(p1, q1, p2, q2, z1.to_bytes(48, "big"), z2.to_bytes(48, "big"), f, e)
    sf, se = ctypes.create_string_buffer(576), ctypes.create_string_buffer(576)
    rs = ht.ht_serial_check(p1, q1, p2, q2, sf, se)
    return rc, f.raw, e.raw, rs, sf.raw, se.raw


def test_gt_pairing_check_matches_serial(ht):
    """Miller loop over precomputed lines with Jacobian G1 points (line scaled by Z^3) +
    cooperative final exponentiation: equal to the serial check for valid and invalid
    equations, for both pair orders (group 0 and 1 of a unit) and Jacobian scalings."""
    rng = random.Random(9)
    g1, g2 = B.G1_GEN, B.G2_GEN
    a, b = rng.randrange(1, B.R), rng.randrange(1, B.R)
    P1, Q1 = B.g1_compress(B.g1_mul(g1, a)), B.g2_compress(B.g2_mul(g2, b))
    good = B.g1_compress(B.g1_mul(g1, a * b % B.R))
    bad = B.g1_compress(B.g1_mul(g1, (a * b + 1) % B.R))
    G2 = B.g2_compress(g2)
    # e(aG1, bG2) == e(abG1, G2): affine points -> the Miller value itself is the serial one
    rc, f, e, rs, sf, se = _check(ht, P1, Q1, good, G2)
    assert rc == 7 and rs == 1 and f == sf and e == se
    rc, f, e, rs, sf, se = _check(ht, P1, Q1, bad, G2)
    assert rc == 1 and rs == 0 and f == sf and e == se
    # Jacobian scalings change the Miller value by an Fq factor, not the final value
    z1, z2 = rng.randrange(1, B.P), rng.randrange(1, B.P)
    rc, f, e, rs, sf, se = _check(ht, P1, Q1, bad, G2, z1, z2)
    assert rc == 1 and e == se and f != sf
    rc, f, e, rs, sf, se = _check(ht, P1, Q1, good, G2, z1, z2)
    assert rc == 7 and e == se


def test_gt_pairing_check_infinity_pairs(ht):
    """An argument at infinity makes its pair contribute 1 (the unit line)."""
    rng = random.Random(10)
    inf1 = bytes([0xC0]) + bytes(47)
    inf2 = bytes([0xC0]) + bytes(95)
    P = B.g1_compress(B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)))
    Q = B.g2_compress(B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)))
    for args, want in (((inf1, Q, inf1, Q), 7), ((P, inf2, inf1, Q), 7), ((P, Q, inf1, Q), 1),
                       ((inf1, Q, P, Q), 1)):
        rc, f, e, rs, sf, se = _check(ht, *args, z1=3, z2=5)
        assert rc == want and e == se and rs == (1 if want == 7 else 0)


def test_binary_gcd_inversion(ht):
    """fq_inv_binary (the final exponentiation's one inversion) on edge values and random ones,
    several lanes at once (lanes finish at different iterations of the wave-uniform loop)."""
    rng = random.Random(11)
    vals = [1, 2, B.P - 1, B.P - 2, 3, 1 << 200, (1 << 380) + 1, 0x10000000000000000]
    vals += [rng.randrange(1, B.P) for _ in range(8)]
    raw = b"".join(v.to_bytes(48, "big") for v in vals)
    out = ctypes.create_string_buffer(48 * len(vals))
    assert ht.ht_fq_inv_binary(len(vals), raw, out) == 0
    for i, v in enumerate(vals):
        assert int.from_bytes(out.raw[48 * i:48 * i + 48], "big") == pow(v, -1, B.P), hex(v)


def test_gt_check_projective_second_pair(ht):
    """SignatureShare form: e(pk, H) e(-G1, sigma) with sigma's lines projective (A, B, C) at
    the fixed affine -G1 — equal to the serial check's final value, accept and reject."""
    rng = random.Random(12)
    sk, h = rng.randrange(1, B.R), rng.randrange(1, B.R)
    pk = B.g1_compress(B.g1_mul(B.G1_GEN, sk))
    H = B.g2_compress(B.g2_mul(B.G2_GEN, h))
    sig = B.g2_compress(B.g2_mul(B.G2_GEN, sk * h % B.R))
    bad = B.g2_compress(B.g2_mul(B.G2_GEN, (sk * h + 7) % B.R))
    g1 = B.g1_compress(B.G1_GEN)
    for s2, want in ((sig, 1), (bad, 0)):
        e = ctypes.create_string_buffer(576)
        rc = ht.ht_gt_check_proj(pk, H, s2, rng.randrange(1, B.P).to_bytes(48, "big"), e)
        sf, se = ctypes.create_string_buffer(576), ctypes.create_string_buffer(576)
        rs = ht.ht_serial_check(pk, H, g1, s2, sf, se)
        assert rc == want and rs == want and e.raw == se.raw


def test_gt_ops_replicated_layout_match_tower(ht):
    """The latency form of the cooperative arithmetic (gt6.h Pos.rep = 3: 18 lanes per value,
    every Fq2 product split over a coefficient's three sub-lanes) gives the tower results, and
    every sub-lane ends with the same value."""
    rng = random.Random(33)
    ht.ht_gt_op_rep.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_char_p, ctypes.c_char_p,
                                ctypes.c_char_p]
    a, b = rand12(rng), rand12(rng)
    c = cyclotomic(ht, rng)
    for code, x in ((0, a), (1, a), (3, a), (4, a), (5, a), (6, a), (8, a), (2, c), (9, c), (7, a)):
        got = ctypes.create_string_buffer(576)
        assert ht.ht_gt_op_rep(code, 3, x, b, got) == 0, code
        assert got.raw == op(ht, "ht_tower_op", code, x, b), code


def test_gt_check_replicated_layout(ht):
    """A whole pairing-product check on two 18-lane groups equals the 6-lane one (Miller value,
    final value, verdict) on a valid pair, a wrong pair and a Jacobian-scaled point."""
    rng = random.Random(34)
    ht.ht_gt_check_rep.argtypes = [ctypes.c_uint32] + [ctypes.c_char_p] * 8
    for valid in (True, False):
        k = rng.randrange(1, B.R)
        h = rng.randrange(1, B.R)
        P1 = B.g1_mul(B.G1_GEN, k)
        Q1 = B.g2_mul(B.G2_GEN, h)
        P2 = B.g1_mul(B.G1_GEN, k * h % B.R if valid else (k * h + 1) % B.R)
        Q2 = B.G2_GEN
        z1 = rng.randrange(1, B.P).to_bytes(48, "big")
        z2 = (1).to_bytes(48, "big")
        args = [B.g1_compress(P1), B.g2_compress(Q1), B.g1_compress(P2), B.g2_compress(Q2), z1, z2]
        f1, e1, f3, e3 = (ctypes.create_string_buffer(576) for _ in range(4))
        r1 = ht.ht_gt_check(*args, f1, e1)
        r3 = ht.ht_gt_check_rep(3, *args, f3, e3)
        assert r1 == r3 and f1.raw == f3.raw and e1.raw == e3.raw
        assert (r3 & 2 != 0) == valid and (r3 & 1) == 1
