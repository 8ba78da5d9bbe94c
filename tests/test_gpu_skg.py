"""GPU parity of the SyncKeyGen checks (src/sync_key_gen.rs:338-498)
through the C ABI (hbtc_skg_check_parts / hbtc_skg_check_acks).

Oracle: oracle/threshold_crypto.py restates BivarCommitment::row / evaluate, Poly::commitment and
coeff_pos; for small t the decisions are compared with the restated equations evaluated
directly (row.commitment() == commit.row(x); commit.evaluate(x, y) == val * G1).  At t = 333
(C5's N = 1000) honest Parts / Acks must pass and single-coefficient / single-value tampering
must be caught (the decision is the mathematical truth of the equation, size-independent).
"""
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from oracle import bls12_381 as B
from oracle import threshold_crypto as TC

pytestmark = pytest.mark.gpu

R = B.R
G1 = B.g1_compress(B.G1_GEN)


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    yield c
    c.close()


def _g1(ctx, vals):
    out, st = ctx.g1_mul(G1, [v % R for v in vals])
    assert not st.any()
    return [bytes(out[48 * i:48 * i + 48]) for i in range(len(vals))]


def _bivar(rng, t):
    """Random symmetric bivariate polynomial: coefficients b[coeff_pos(i, j)], i <= j."""
    return [rng.randrange(R) for _ in range((t + 1) * (t + 2) // 2)]


def _bivar_eval(b, t, x, y):
    return sum(b[TC.coeff_pos(i, j)] * pow(x, i, R) * pow(y, j, R)
               for i in range(t + 1) for j in range(t + 1)) % R


def test_parts_and_acks_small_vs_oracle(ctx):
    rng = random.Random(2024)
    t, n_nodes, our = 3, 10, 4
    x = our + 1
    n_parts = 6
    polys = [_bivar(rng, t) for _ in range(n_parts)]
    commits = [_g1(ctx, b) for b in polys]
    rows = [TC.bivar_poly_row(b, t, x) for b in polys]
    # corruptions: part 1 row coefficient tampered, part 2 one commitment point replaced,
    # part 3 a commitment point with an invalid encoding, part 4 a row coefficient >= r
    rows[1][2] = (rows[1][2] + 1) % R
    commits[2][5] = _g1(ctx, [polys[2][5] + 7])[0]
    bad = bytearray(commits[3][0])
    bad[0] &= 0x7F
    commits[3][0] = bytes(bad)
    rows[4][0] = R + 5
    st = ctx.skg_check_parts(t, our, [p for c in commits for p in c], rows)
    assert [N.STATUS_NAMES[int(s)] for s in st] == ["ACCEPT", "REJECT", "REJECT", "DECODE_ERR",
                                                    "REJECT", "ACCEPT"]
    # the oracle's direct restatement agrees on the well-formed ones
    for p in (0, 1, 2, 5):
        cm = [B.g1_decompress(q) for q in commits[p]]
        lhs = [B.g1_compress(q) for q in TC.bivar_commitment_row(cm, t, x)]
        rhs = [B.g1_compress(q) for q in TC.commitment([v % R for v in rows[p]])]
        assert (lhs == rhs) == (st[p] == N.ACCEPT)

    # Acks: values val = b(x, y_sender); some tampered; parts 0, 5 have verified rows, parts 1
    # and 2 do not (their Acks go through the MSM combination + exact fallback)
    row_ok = [1 if s == N.ACCEPT else 0 for s in st]
    ack_part, ack_sender, vals, expect = [], [], [], []
    for p in (0, 1, 2, 5):
        for s in range(n_nodes):
            v = _bivar_eval(polys[p], t, x, s + 1)
            tamper = (p, s) in {(0, 3), (1, 0), (1, 7), (5, 9)}
            if tamper:
                v = (v + 11) % R
            ack_part.append(p)
            ack_sender.append(s)
            vals.append(v)
            # part 2's commitment has one wrong point: its evaluate differs from b(x, y)
            cm = [B.g1_decompress(q) for q in commits[p]]
            want = B.g1_compress(TC.bivar_commitment_evaluate(cm, t, x, s + 1))
            expect.append(N.ACCEPT if want == _g1(ctx, [v])[0] else N.REJECT)
    ack_part.append(0)
    ack_sender.append(1)
    vals.append(R + 1)  # not a canonical Fr: ValueDeserialization
    expect.append(N.DECODE_ERR)
    ast = ctx.skg_check_acks(t, our, [p for c in commits for p in c],
                             [[v % R for v in r] for r in rows], row_ok, ack_part, ack_sender,
                             vals)
    assert list(ast) == expect
    assert expect.count(N.REJECT) >= 4 + 9  # part 2: every Ack is off (one bad commitment point)


def test_acks_without_rows_all_valid(ctx):
    """Observer-like view of one Part without a verified row: the combination passes."""
    rng = random.Random(77)
    t, our = 4, 2
    b = _bivar(rng, t)
    commit = _g1(ctx, b)
    senders = list(range(12))
    vals = [_bivar_eval(b, t, our + 1, s + 1) for s in senders]
    st = ctx.skg_check_acks(t, our, commit, None, [0], [0] * len(senders), senders, vals)
    assert list(st) == [N.ACCEPT] * len(senders)


def test_c5_scale_part_and_acks(ctx):
    """t = 333 (N = 1000): 2 Parts of 55,945 commitment points, honest and one tampered row
    coefficient; 1000 Acks against a verified row (scalar path) with 3 tampered values."""
    rng = random.Random(5)
    t, our = 333, 17
    x = our + 1
    polys = [_bivar(rng, t) for _ in range(2)]
    commits = [p for b in polys for p in _g1(ctx, b)]
    rows = [TC.bivar_poly_row(b, t, x) for b in polys]
    rows[1][200] = (rows[1][200] + 1) % R
    st = ctx.skg_check_parts(t, our, commits, rows)
    assert list(st) == [N.ACCEPT, N.REJECT]
    senders = list(range(1000))
    vals = [TC.poly_evaluate(rows[0], s + 1) for s in senders]
    bad = {5, 500, 999}
    for s in bad:
        vals[s] = (vals[s] + 1) % R
    ast = ctx.skg_check_acks(t, our, commits, rows, [1, 0], [0] * 1000, senders, vals)
    assert [i for i, s in enumerate(ast) if s != N.ACCEPT] == sorted(bad)
