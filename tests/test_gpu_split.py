"""The split levels of the RLC DecryptionShare path (hbtc_check.hip k_chk_split): a failing tile
that single-error location cannot resolve is split by checking its LEFT child and deriving the
right one (T_R = T_X / T_L, U_R = U_X / (W_L^(2 alpha) T_L^beta)), down to eighths and then the
exact leaf checks.  Error patterns aimed at every path — both errors in the left half, both in
the derived right half (location under alpha = 2, 4, 8), one per half, one per quarter, two in
one eighth (leaves, also at the deepest derived node), three in one quarter, a cancelling pair,
every share wrong, ragged tiles whose right children are short or empty — must give exactly the
per-share decisions under every check schedule, with the split levels (default) and without
(HBTC_SPLIT=0: the round-3 halves / sub-tile levels), at 64- and 128-bit RLC scalars.
Reference: PublicKeyShare::verify_decryption_share, /root/reference/src/threshold_decryption.rs:159."""
import os
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from tests.test_gpu_parity import R, _keyset, b, load

pytestmark = pytest.mark.gpu

# (tile size, wrong positions inside the tile, cancelling pair or None)
PATTERNS = [
    (64, [3, 20], None),           # both in the left half, one per quarter
    (64, [35, 60], None),          # both in the derived right half
    (64, [5, 40], None),           # one per half
    (64, [1, 2], None),            # one eighth (left path down to the leaves)
    (64, [62, 63], None),          # one eighth at the deepest derived node
    (64, [50, 60, 61], None),      # three in quarter 3: eighth 6 located, eighth 7 to leaves
    (64, [0, 16, 32, 48], None),   # one per quarter
    (64, [], (10, 11)),            # a cancelling pair inside one eighth
    (64, [], (8, 40)),             # a cancelling pair across halves
    (64, list(range(64)), None),   # every share wrong
    (64, [7, 15, 23, 31, 39, 47, 55, 63], None),  # the last share of every eighth
    (50, [33, 49], None),          # ragged: right half of 18, quarter 3 of 2
    (37, [2, 3, 36], None),        # ragged: right half of 5
    (9, [0, 8], None),             # ragged: a 9-share tile
    (33, [31, 32], None),          # ragged: the right half is one share
]


def _batch(ctx, rng):
    n = 70
    f, coeffs, sks, pk = _keyset(ctx, rng, n)
    codec = load("codec.json")
    g1, g2 = b(codec["g1_generator"]), b(codec["g2_generator"])
    counts = [p[0] for p in PATTERNS]
    n_ct = len(counts)
    rs = [rng.randrange(1, R) for _ in range(n_ct)]
    hs = [rng.randrange(1, R) for _ in range(n_ct)]
    H, _ = ctx.g2_mul(g2, hs)
    w, _ = ctx.g2_mul(g2, [r * h % R for r, h in zip(rs, hs)])
    idx, scal, exp = [], [], []
    for k, (c, wrong, pair) in enumerate(PATTERNS):
        base = len(idx)
        for j in range(c):
            i = (j * 13 + 5 * k) % n
            idx.append(i)
            scal.append(sks[i] * rs[k] % R)
            exp.append(N.ACCEPT)
        for j in wrong:
            scal[base + j] = (scal[base + j] + rng.randrange(1, 1 << 40)) % R
            exp[base + j] = N.REJECT
        if pair:
            d = rng.randrange(1, R)
            scal[base + pair[0]] = (scal[base + pair[0]] + d) % R
            scal[base + pair[1]] = (scal[base + pair[1]] - d) % R
            exp[base + pair[0]] = exp[base + pair[1]] = N.REJECT
    shares, st = ctx.g1_mul(g1, scal)
    assert not st.any()
    return pk, H, w, counts, idx, shares, np.asarray(exp, np.int32)


@pytest.mark.parametrize("split", ["1", "0"])
def test_split_levels_equal_per_share_decisions(split):
    old = os.environ.get("HBTC_SPLIT")
    os.environ["HBTC_SPLIT"] = split
    try:
        ctx = N.Context(0)  # reads HBTC_SPLIT at creation
        ctx.set_exact_below(0)
    finally:
        if old is None:
            del os.environ["HBTC_SPLIT"]
        else:
            os.environ["HBTC_SPLIT"] = old
    try:
        pk, H, w, counts, idx, shares, exp = _batch(ctx, random.Random(515))
        ks, _ = ctx.keyset_load(pk)
        ctx.set_verify_mode(N.MODE_PER_SHARE)
        st_ref = ctx.verify_dec_shares(ks, H, w, counts, idx, shares)
        assert (st_ref == exp).all(), np.nonzero(st_ref != exp)
        ctx.set_verify_mode(N.MODE_RLC)
        for bits in (128, 64):
            ctx.set_rlc_bits(bits)
            for sched in (N.CHECK_AUTO, N.CHECK_PLAIN_FIRST, N.CHECK_PAIR_SUBS, N.CHECK_PAIR_LEAVES):
                ctx.set_check_schedule(sched)
                st = ctx.verify_dec_shares(ks, H, w, counts, idx, shares)
                assert (st == exp).all(), (split, bits, sched, np.nonzero(st != exp))
    finally:
        ctx.close()


def test_split_levels_cut_leaf_checks():
    """The split levels (the plain-first schedule's: the paired ones keep their one sub-tile
    level) resolve tiles whose wrong shares sit in different eighths without exact leaf checks:
    only the eighths holding >= 2 wrong shares reach them."""
    ctx = N.Context(0)
    ctx.set_exact_below(0)
    try:
        pk, H, w, counts, idx, shares, exp = _batch(ctx, random.Random(516))
        ks, _ = ctx.keyset_load(pk)
        ctx.set_verify_mode(N.MODE_RLC)
        ctx.set_check_schedule(N.CHECK_PLAIN_FIRST)
        ctx.timing_enable(True)
        st = ctx.verify_dec_shares(ks, H, w, counts, idx, shares)
        assert (st == exp).all()
        assert all(ctx.timing_read("chk_split%d" % lvl)[1] >= 1 for lvl in (1, 2, 3))
        leaves = ctx.rlc_last_leaves()
        # the eighths with >= 2 wrong shares, 8 shares each: (1, 2), (62, 63), (60, 61), the pair
        # (10, 11), (2, 3) of the 37-share tile, the 8 eighths of the all-wrong tile; (0, 8) of the
        # 9-share tile and (31, 32) of the 33-share tile straddle eighths (located, no leaves)
        assert leaves == 8 * 13, leaves
    finally:
        ctx.close()
