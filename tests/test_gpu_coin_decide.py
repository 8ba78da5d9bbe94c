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


def _golden_c1_instances(c):
    """hbtc_coin_decide instances built from the C1 coin fixture (tests/golden/c1_coin.json, the
    threshold_crypto restatement's vectors): per instance the items, and the expected item
    statuses, coin status, combined signature and parity."""
    it = {i["name"]: i for i in c["items"]}
    comb = {x["name"]: x for x in c["combines"]}
    rejects = [n for n in it if it[n]["expected"] != "ACCEPT"]
    insts = [
        # every fixture item in fixture order: the first t ACCEPTed are nodes 0..3
        ("all", list(it), "ACCEPT", comb["first_t"]),
        # every rejected / undecodable item first, then nodes 6..9: the combine skips them all
        ("rejects_then_last_t", rejects + ["valid_%d" % i for i in range(6, 10)], "ACCEPT", comb["last_t"]),
        # a wrong share in the middle of the first t + 1 (the speculation's leave-one-out subset)
        ("one_wrong_first", ["valid_0", "valid_1", "wrong_message", "valid_2", "valid_3", "valid_4"],
         "ACCEPT", comb["first_t"]),
        ("not_enough", ["valid_0", "wrong_key", "valid_1", "identity", "valid_2", "enc_not_in_subgroup"],
         "NOT_ENOUGH_SHARES", comb["not_enough"]),
        ("duplicate", ["valid_0", "valid_0", "valid_1", "valid_2", "valid_3"], "DUPLICATE_ENTRY",
         comb["duplicate"]),
    ]
    return it, insts


def test_coin_decide_golden_c1():
    """hbtc_coin_decide against the C1 coin fixture: item statuses, the coin status, the combined
    signature's bytes and its parity bit equal the threshold_crypto restatement's vectors
    (coin.rs:151 / :185-191 / :173 / :192-197), with the speculation on and off."""
    c = json.load(open(os.path.join(HERE, "golden", "c1_coin.json")))
    assert c["master_verify"] is True
    b = bytes.fromhex
    it, insts = _golden_c1_instances(c)
    counts = [len(names) for _, names, _, _ in insts]
    idx = [it[n]["idx"] for _, names, _, _ in insts for n in names]
    sigs = [b(it[n]["sig"]) for _, names, _, _ in insts for n in names]
    H = [b(c["H"])] * len(insts)
    want_st = [it[n]["expected"] for _, names, _, _ in insts for n in names]
    for spec in ("1", "0"):
        old = os.environ.get("HBTC_COIN_SPEC")
        os.environ["HBTC_COIN_SPEC"] = spec
        try:
            cx = N.Context(0)
            try:
                ks, nbad = cx.keyset_load([b(p) for p in c["pk_shares"]])
                assert nbad == 0
                cx.keyset_set_master(ks, b(c["master_pk"]))
                st, out, par, cst = cx.coin_decide(ks, H, counts, idx, sigs, c["t"])
                # the single-coin form hbbft calls once per coin (c1: one instance per call)
                one = cx.coin_decide(ks, H[:1], counts[:1], idx[:counts[0]], sigs[:counts[0]], c["t"])
            finally:
                cx.close()
        finally:
            if old is None:
                os.environ.pop("HBTC_COIN_SPEC", None)
            else:
                os.environ["HBTC_COIN_SPEC"] = old
        assert [N.STATUS_NAMES[int(s)] for s in st] == want_st, spec
        for k, (name, _, want_coin, cmb) in enumerate(insts):
            assert N.STATUS_NAMES[int(cst[k])] == want_coin == cmb["expected"], (spec, name)
            if want_coin == "ACCEPT":
                assert out[k].hex() == cmb["sig"], (spec, name)
                assert int(par[k]) == cmb["parity"], (spec, name)
        assert [N.STATUS_NAMES[int(s)] for s in one[0]] == want_st[:counts[0]], spec
        assert one[1][0].hex() == insts[0][3]["sig"] and int(one[2][0]) == insts[0][3]["parity"], spec
        assert int(one[3][0]) == N.ACCEPT, spec
