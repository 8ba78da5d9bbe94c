"""GPU parity of the pair-batch RLC path (hbbft_amd/csrc/hbtc_pb.hip): e(A_i, Q_i) == e(G1, W_i)
for a batch, as hbtc_verify_ciphertexts (Ciphertext::verify: e(G1, w) == e(u, H)), hbtc_verify_sigs
(PublicKey::verify: e(pk, H) == e(G1, sigma)) and hbtc_decrypt use it.  The RLC decisions must
equal the per-share path's (one exact pairing check per item, k_pair_verify) on valid items,
wrong ones, bad encodings and points at infinity, inside one 64-item tile, across tiles and
across chunk boundaries (a context with 4096-item chunks)."""
import json
import os
import random

import numpy as np
import pytest

from hbbft_amd import _native as N

pytestmark = pytest.mark.gpu

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
GOLDEN = os.path.join(os.path.dirname(__file__), "golden")
G1_INF = bytes([0xC0]) + bytes(47)
G2_INF = bytes([0xC0]) + bytes(95)


def _gens():
    with open(os.path.join(GOLDEN, "codec.json")) as fh:
        d = json.load(fh)
    return bytes.fromhex(d["g1_generator"]), bytes.fromhex(d["g2_generator"])


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    c.set_exact_below(0)  # this module tests the pair-batch path: small calls batch too
    yield c
    c.close()


def _split(buf, size):
    buf = bytes(buf)
    return [buf[i:i + size] for i in range(0, len(buf), size)]


def _ct_batch(ctx, rng, n, n_distinct=96):
    """n ciphertext triples (u, H, w) built from n_distinct valid ones, then damaged: wrong w,
    bad encodings of u / H / w, u = O, H = O (valid iff w = O), a pair whose errors cancel."""
    g1, g2 = _gens()
    rs = [rng.randrange(1, R) for _ in range(n_distinct)]
    hs = [rng.randrange(1, R) for _ in range(n_distinct)]
    u = _split(ctx.g1_mul(g1, rs)[0], 48)
    H = _split(ctx.g2_mul(g2, hs)[0], 96)
    w = _split(ctx.g2_mul(g2, [r * h % R for r, h in zip(rs, hs)])[0], 96)
    pick = [rng.randrange(n_distinct) for _ in range(n)]
    us, Hs, ws = [u[p] for p in pick], [H[p] for p in pick], [w[p] for p in pick]
    k = max(1, n // 100)
    wrong = rng.sample(range(n), k)
    deltas = [rng.randrange(1, 1 << 20) for _ in wrong]
    bad_w = _split(ctx.g2_mul(g2, [(rs[pick[i]] * hs[pick[i]] + d) % R for i, d in zip(wrong, deltas)])[0], 96)
    for i, bw in zip(wrong, bad_w):
        ws[i] = bw
    if n > 20:  # two wrong items whose errors cancel in an unweighted sum
        d = rng.randrange(1, R)
        a, b = 10, 11
        ws[a], ws[b] = _split(ctx.g2_mul(g2, [(rs[pick[a]] * hs[pick[a]] + d) % R,
                                              (rs[pick[b]] * hs[pick[b]] - d) % R])[0], 96)
        us[12] = bytes([us[12][0] & 0x7F]) + us[12][1:]  # encodings pairing 0.14 refuses
        Hs[13] = bytes([Hs[13][0] & 0x7F]) + Hs[13][1:]
        ws[14] = bytes([ws[14][0] & 0x7F]) + ws[14][1:]
        us[15], ws[15] = G1_INF, G2_INF  # e(O, H) = 1 = e(G1, O): valid
        Hs[16], ws[16] = G2_INF, G2_INF  # e(u, O) = 1 = e(G1, O): valid
        Hs[17] = G2_INF                  # e(u, O) = 1 != e(G1, w): wrong
    return us, Hs, ws


@pytest.mark.parametrize("n", [1, 40, 64, 200, 65536 + 130])
def test_verify_ciphertexts_rlc_equals_per_share(ctx, n):
    """Ciphertext::verify by pair-batch RLC equals the per-item check (one chunk: the default
    chunk is 2^18 items)."""
    _ct_rlc_equals_per_share(ctx, n)


def test_verify_ciphertexts_across_chunks():
    """The multi-chunk path of pb_verify_dev: a context with 4096-item chunks
    (HBTC_PB_CHUNK) verifies 3 x 4096 + 130 ciphertexts in four chunks — base offsets into the
    item and status arrays, a fresh key per chunk, workspace reused across chunks, each chunk's
    exact-check list — with the same decisions as the per-item path, at 64- and 128-bit scalars;
    then hbtc_trim_workspace frees the cache and the context still works."""
    os.environ["HBTC_PB_CHUNK"] = "4096"
    try:
        c = N.Context(0)
    finally:
        del os.environ["HBTC_PB_CHUNK"]
    c.set_exact_below(0)
    try:
        _ct_rlc_equals_per_share(c, 3 * 4096 + 130, extra_bad=(4095, 4096, 8191, 12287, 12290))
        c.trim_workspace()
        _ct_rlc_equals_per_share(c, 200)
    finally:
        c.close()


def _ct_rlc_equals_per_share(ctx, n, extra_bad=()):
    rng = random.Random(n + 5)
    us, Hs, ws = _ct_batch(ctx, rng, n)
    for i in extra_bad:  # wrong w at chunk edges
        us[i], ws[i] = us[i], ws[(i + 1) % n]
    ctx.set_verify_mode(N.MODE_PER_SHARE)
    ref = ctx.verify_ciphertexts(us, Hs, ws)
    for i in extra_bad:
        assert ref[i] == N.REJECT, i
    ctx.set_verify_mode(N.MODE_RLC)
    for bits in (64, 128):
        ctx.set_rlc_bits(bits)
        try:
            st = ctx.verify_ciphertexts(us, Hs, ws)
        finally:
            ctx.set_rlc_bits(128)  # the library default
        assert (st == ref).all(), (bits, np.nonzero(st != ref)[0][:20])
    if n > 20:
        assert ref[10] == N.REJECT and ref[11] == N.REJECT
        assert ref[12] == N.DECODE_ERR and ref[13] == N.DECODE_ERR and ref[14] == N.DECODE_ERR
        assert ref[15] == N.ACCEPT and ref[16] == N.ACCEPT and ref[17] == N.REJECT
        assert (ref == N.ACCEPT).sum() >= n - n // 100 - 10


def test_verify_sigs_rlc_equals_per_share(ctx):
    """PublicKey::verify batches (votes, combined coin signatures): e(pk, H) == e(G1, sigma)."""
    rng = random.Random(77)
    g1, g2 = _gens()
    n = 150
    sks = [rng.randrange(1, R) for _ in range(n)]
    hs = [rng.randrange(1, R) for _ in range(n)]
    pk = _split(ctx.g1_mul(g1, sks)[0], 48)
    H = _split(ctx.g2_mul(g2, hs)[0], 96)
    sc = [s * h % R for s, h in zip(sks, hs)]
    for i in (3, 70, 71, 149):
        sc[i] = (sc[i] + 1) % R
    sig = _split(ctx.g2_mul(g2, sc)[0], 96)
    sig[5] = bytes([sig[5][0] & 0x7F]) + sig[5][1:]
    ctx.set_verify_mode(N.MODE_PER_SHARE)
    ref = ctx.verify_sigs(pk, H, sig)
    ctx.set_verify_mode(N.MODE_RLC)
    st = ctx.verify_sigs(pk, H, sig)
    assert (st == ref).all(), np.nonzero(st != ref)
    assert [int(x) for x in np.nonzero(ref == N.REJECT)[0]] == [3, 70, 71, 149]
    assert ref[5] == N.DECODE_ERR


@pytest.mark.parametrize("n", [1, 40, 255])
def test_small_pair_calls_take_exact_leaf_checks(n):
    """With the default hbtc_set_exact_below (256), Ciphertext::verify calls of fewer items run
    as exact SignatureShare-form checks (A decoded, Q's line tables, W decoded and checked by the
    cooperative leaf kernels): the per-item decisions of k_pair_verify on wrong w, bad encodings
    of u / H / w, u = O, H = O, a cancelling pair; no pair-batch launch."""
    c = N.Context(0)
    c.timing_enable(True)
    try:
        us, Hs, ws = _ct_batch(c, random.Random(n + 11), n)
        c.set_verify_mode(N.MODE_PER_SHARE)
        ref = c.verify_ciphertexts(us, Hs, ws)
        c.set_verify_mode(N.MODE_RLC)
        c.timing_reset()
        st = c.verify_ciphertexts(us, Hs, ws)
        assert (st == ref).all(), (n, np.nonzero(st != ref))
        assert c.timing_read("pb_items")[1] == 0 and c.timing_read("chk_leaves")[1] >= 1
        if n > 20:
            assert ref[13] == N.DECODE_ERR and ref[15] == N.ACCEPT and ref[16] == N.ACCEPT
            assert ref[17] == N.REJECT and ref[10] == N.REJECT and ref[11] == N.REJECT
    finally:
        c.close()
