"""GPU parity of hbtc_prepare_g2 (per-instance G2 tables built ahead of the shares: a coin's H
when the Coin is created, /root/reference/src/binary_agreement/binary_agreement.rs:320; a
ciphertext's H and w at set_ciphertext, /root/reference/src/threshold_decryption.rs:94-113).

Bar: every verification output of a call whose G2 arguments are prepared is bit-equal to the
same call unprepared (and to the golden fixtures where they exist), the prepared tables are
really the ones used (the call's `prepare_cached` timing family, no `prepare` launch), a bad
encoding is reported as unprepared, and unprepare / re-prepare keeps working.
"""
import json
import os

import numpy as np
import pytest

from hbbft_amd import _native as N

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
b = bytes.fromhex


def fx(name):
    with open(os.path.join(HERE, "golden", name)) as fh:
        return json.load(fh)


def _fresh(spec=None):
    old = os.environ.get("HBTC_COIN_SPEC")
    if spec is not None:
        os.environ["HBTC_COIN_SPEC"] = spec
    try:
        return N.Context(0)
    finally:
        if spec is not None:
            if old is None:
                os.environ.pop("HBTC_COIN_SPEC", None)
            else:
                os.environ["HBTC_COIN_SPEC"] = old


def _families(ctx, fams):
    return {f: ctx.timing_read(f)[1] for f in fams}


@pytest.mark.parametrize("spec", ["1", "0"])
def test_prepared_coin_equals_unprepared_and_golden(spec):
    c = fx("c1_coin.json")
    items = c["items"]
    H = [b(c["H"])]
    idx = [i["idx"] for i in items]
    sigs = [b(i["sig"]) for i in items]
    want = [i["expected"] for i in items]
    outs = []
    for prepared in (False, True):
        ctx = _fresh(spec)
        try:
            ks, _ = ctx.keyset_load([b(p) for p in c["pk_shares"]])
            ctx.keyset_set_master(ks, b(c["master_pk"]))
            if prepared:
                assert list(ctx.prepare_g2(H)) == [N.ACCEPT]
                assert ctx.prepared_g2_count() == 1
            ctx.timing_enable(True)
            ctx.timing_reset()
            st = ctx.verify_sig_shares(ks, H, [len(items)], idx, sigs)
            got = ctx.coin_decide(ks, H, [len(items)], idx, sigs, c["t"])
            fam = _families(ctx, ("prepare", "prepare_cached"))
            if prepared:
                assert fam["prepare"] == 0 and fam["prepare_cached"] >= 2, fam
            else:
                assert fam["prepare"] >= 2 and fam["prepare_cached"] == 0, fam
            outs.append((list(st), list(got[0]), got[1], list(got[2]), list(got[3])))
        finally:
            ctx.close()
    assert outs[0] == outs[1]
    assert [N.STATUS_NAMES[int(s)] for s in outs[1][0]] == want
    comb = c["combines"][0]
    assert outs[1][2][0].hex() == comb["sig"] and outs[1][3][0] == comb["parity"] and outs[1][4][0] == N.ACCEPT


def test_prepared_dec_shares_equal_unprepared_and_golden():
    d = fx("c1_dec.json")
    items = d["items"]
    H, w = [b(d["H"])], [b(d["w"])]
    idx = [i["idx"] for i in items]
    shares = [b(i["share"]) for i in items]
    res = []
    for prepared in (False, True):
        ctx = N.Context(0)
        try:
            ks, _ = ctx.keyset_load([b(p) for p in d["pk_shares"]])
            if prepared:
                assert list(ctx.prepare_g2(H + w)) == [N.ACCEPT, N.ACCEPT]
            ctx.timing_enable(True)
            ctx.timing_reset()
            st = ctx.verify_dec_shares(ks, H, w, [len(items)], idx, shares)
            fam = _families(ctx, ("prepare", "prepare_cached"))
            assert (fam["prepare_cached"] >= 1) == prepared and (fam["prepare"] == 0) == prepared, fam
            res.append(list(st))
        finally:
            ctx.close()
    assert res[0] == res[1]
    assert [N.STATUS_NAMES[int(s)] for s in res[1]] == [i["expected"] for i in items]


def test_partly_prepared_and_bad_points():
    """A call with one unprepared argument builds all of its tables (same outputs); a point
    that fails to decode is prepared as DECODE_ERR and its instance reports the same statuses
    as unprepared; unprepare drops entries and a second prepare rebuilds them."""
    c = fx("c1_coin.json")
    codec = fx("codec.json")
    bad = b(codec["g2_bad"][0]["enc"])
    items = [i for i in c["items"] if i["name"].startswith("valid")]
    idx = [i["idx"] for i in items]
    sigs = [b(i["sig"]) for i in items]
    H = [b(c["H"]), bad]
    counts = [len(items) // 2, len(items) - len(items) // 2]
    ref_ctx = N.Context(0)
    try:
        ks, _ = ref_ctx.keyset_load([b(p) for p in c["pk_shares"]])
        ref = list(ref_ctx.verify_sig_shares(ks, H, counts, idx, sigs))
    finally:
        ref_ctx.close()
    ctx = N.Context(0)
    try:
        ks, _ = ctx.keyset_load([b(p) for p in c["pk_shares"]])
        assert list(ctx.prepare_g2([H[0]])) == [N.ACCEPT]
        ctx.timing_enable(True)
        ctx.timing_reset()
        assert list(ctx.verify_sig_shares(ks, H, counts, idx, sigs)) == ref  # only H[0] prepared
        assert _families(ctx, ("prepare",))["prepare"] >= 1
        st = ctx.prepare_g2(H)
        assert list(st) == [N.ACCEPT, N.DECODE_ERR] and ctx.prepared_g2_count() == 2
        ctx.timing_reset()
        assert list(ctx.verify_sig_shares(ks, H, counts, idx, sigs)) == ref
        assert _families(ctx, ("prepare",))["prepare"] == 0
        ctx.unprepare_g2(H)
        assert ctx.prepared_g2_count() == 0
        assert list(ctx.prepare_g2(H[::-1])) == [N.DECODE_ERR, N.ACCEPT]
        assert list(ctx.verify_sig_shares(ks, H, counts, idx, sigs)) == ref
    finally:
        ctx.close()
    assert all(s != N.ACCEPT for s in ref[counts[0]:])  # the bad H's instance accepts nothing
