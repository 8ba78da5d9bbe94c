"""GPU parity of hbtc_coin_decide (one Threshold Coin round in one call, src/coin.rs:149-207)
against the separate entry points it replaces: hbtc_verify_sig_shares (PublicKeyShare::verify,
coin.rs:151), hbtc_combine_sigs over the first t ACCEPTed shares (combine_signatures,
coin.rs:185-191) and hbtc_verify_sigs against the master key (PublicKey::verify, coin.rs:192-197).

Patterns: every share valid; one wrong share among the first t (the speculation's leave-one-out
subset); the wrong share right after them; two wrong among the first t + 1 (the status-driven
combine); fewer than t valid (NOT_ENOUGH_SHARES); bad encodings; an unknown sender; a repeated
node index (DUPLICATE_ENTRY); and a key set whose master key does not match its shares (the
combined signature fails PublicKey::verify: REJECT).  With the speculation on and off, and with a
batch too large to speculate.  Bar: identical statuses, bytes and parity bits.
"""
import json
import os
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from oracle import bls12_381 as B

pytestmark = pytest.mark.gpu

R = B.R
HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    yield c
    c.close()


def _instances(rng, n, t, n_inst, sks, hs, bad2):
    """counts, idx, sig scalars / overrides per pattern (cycled over the instances)."""
    patterns = ["valid", "one_wrong_first", "wrong_after", "two_wrong", "short", "bad_enc",
                "unknown", "dup"]
    counts, idx, scal, edits, kinds = [], [], [], [], []
    for k in range(n_inst):
        kind = patterns[k % len(patterns)]
        ids = list(range(n))
        if kind == "unknown":
            ids = [0, n + 5] + list(range(1, n))  # sender n + 5 is not in the key set
        if kind == "dup":
            ids = [0, 1, 1] + list(range(2, n))
        wrong = set()
        if kind == "one_wrong_first":
            wrong = {min(2, t - 1)}
        elif kind == "wrong_after":
            wrong = {t}
        elif kind == "two_wrong":
            wrong = {0, min(1, t)} if t > 1 else {0, 1}
        elif kind == "short":
            wrong = set(range(n - t + 1))  # only t - 1 valid shares
        base = len(scal)
        for j, i in enumerate(ids):
            s = sks[i % len(sks)] * hs[k] % R
            scal.append((s + 1) % R if j in wrong else s)
        if kind == "bad_enc":
            edits.append((base + 1, bad2[k % len(bad2)]))
        counts.append(len(ids))
        idx += ids
        kinds.append(kind)
    return counts, idx, scal, edits, kinds


def _reference(ctx, ks, H, counts, idx, sigs, t, mpk):
    """The separate entry points, as hbbft calls them per share / per combine / per check."""
    st = ctx.verify_sig_shares(ks, H, counts, idx, sigs)
    sel_counts, sel_idx, sel_sigs = [], [], []
    pos = 0
    for c in counts:
        acc = [j for j in range(pos, pos + c) if st[j] == N.ACCEPT][:t]
        sel_counts.append(len(acc))
        sel_idx += [idx[j] for j in acc]
        sel_sigs += [sigs[j] for j in acc]
        pos += c
    out, par, cst = ctx.combine_sigs(sel_counts, sel_idx, sel_sigs, t)
    coin = []
    for k in range(len(counts)):
        if cst[k] != N.ACCEPT:
            coin.append(int(cst[k]))
            continue
        ok = ctx.verify_sigs([mpk], [H[k]], [out[k]])
        coin.append(int(ok[0]))
    return st, out, par, cst, coin


@pytest.mark.parametrize("n,t,n_inst", [(10, 4, 8), (10, 1, 8), (7, 3, 16), (10, 4, 64)])
def test_coin_decide_equals_separate_calls(ctx, n, t, n_inst):
    rng = random.Random(31 * n + t + n_inst)
    poly = [rng.randrange(1, R) for _ in range(t)]
    sks = [sum(c * pow(i + 1, e, R) for e, c in enumerate(poly)) % R for i in range(n)]
    g1 = B.g1_compress(B.G1_GEN)
    g2 = B.g2_compress(B.G2_GEN)
    pk, st = ctx.g1_mul(g1, sks)
    assert not st.any()
    mpk, _ = ctx.g1_mul(g1, [poly[0]])
    wrong_mpk, _ = ctx.g1_mul(g1, [(poly[0] + 1) % R])
    hs = [rng.randrange(1, R) for _ in range(n_inst)]
    Hs, _ = ctx.g2_mul(g2, hs)
    H = [bytes(Hs[96 * k:96 * k + 96]) for k in range(n_inst)]
    codec = json.load(open(os.path.join(HERE, "golden", "codec.json")))
    bad2 = [bytes.fromhex(x["enc"]) for x in codec["g2_bad"]]
    counts, idx, scal, edits, kinds = _instances(rng, n, t, n_inst, sks, hs, bad2)
    # sigma_i = sk_i * H_k = (sk_i h_k) G2
    sg, st2 = ctx.g2_mul(g2, scal)
    assert not st2.any()
    sigs = [bytes(sg[96 * i:96 * i + 96]) for i in range(len(scal))]
    for pos, enc in edits:
        sigs[pos] = enc
    ks, nbad = ctx.keyset_load(pk)
    assert nbad == 0
    try:
        for master in (bytes(mpk), bytes(wrong_mpk)):
            ctx.keyset_set_master(ks, master)
            ref = _reference(ctx, ks, H, counts, idx, sigs, t, master)
            for spec in ("1", "0"):
                old = os.environ.get("HBTC_COIN_SPEC")
                os.environ["HBTC_COIN_SPEC"] = spec
                try:
                    c2 = N.Context(0)
                    try:
                        ks2, _ = c2.keyset_load(pk)
                        c2.keyset_set_master(ks2, master)
                        got = c2.coin_decide(ks2, H, counts, idx, sigs, t)
                    finally:
                        c2.close()
                finally:
                    if old is None:
                        os.environ.pop("HBTC_COIN_SPEC", None)
                    else:
                        os.environ["HBTC_COIN_SPEC"] = old
                st_g, out_g, par_g, coin_g = got
                assert list(st_g) == list(ref[0]), (spec, kinds)
                assert out_g == ref[1], spec
                assert list(par_g) == list(ref[2]), spec
                assert list(coin_g) == ref[4], (spec, list(coin_g), ref[4], kinds)
            if master == bytes(mpk):
                # the construction: every instance with t valid shares combines to master * h_k
                for k, kind in enumerate(kinds):
                    if ref[3][k] == N.ACCEPT:
                        assert ref[4][k] == N.ACCEPT
                        want, _ = ctx.g2_mul(g2, [poly[0] * hs[k] % R])
                        assert ref[1][k] == bytes(want), kind
            else:
                assert all(c != N.ACCEPT for c in ref[4])
    finally:
        ctx.keyset_free(ks)


def test_coin_decide_needs_master(ctx):
    g1 = B.g1_compress(B.G1_GEN)
    pk, _ = ctx.g1_mul(g1, [1, 2, 3, 4])
    ks, _ = ctx.keyset_load(pk)
    try:
        with pytest.raises(N.HbtcError):
            ctx.coin_decide(ks, [B.g2_compress(B.G2_GEN)], [1], [0], [B.g2_compress(B.G2_GEN)], 1)
        bad = bytes.fromhex(json.load(open(os.path.join(HERE, "golden", "codec.json")))["g1_bad"][4]["enc"])
        with pytest.raises(N.HbtcError):
            ctx.keyset_set_master(ks, bad)
    finally:
        ctx.keyset_free(ks)
    assert np.int32(N.ACCEPT) == 0
