"""The batch queues (hbbft_amd/protocol.py) against the reference's sequential decision rules
(oracle/hbbft_rules.py, a restatement of src/coin.rs and src/threshold_decryption.rs): random
arrival orders, corrupted shares, unknown senders, duplicates, messages after termination and
several flushes per epoch must give exactly the reference's faults, errors and outputs.

CPU variant: the queues drive a test double whose crypto is the C oracle (the replay logic is
host logic).  GPU variant (-m gpu): the queues drive the real HIP library."""
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from hbbft_amd import protocol as P
from oracle import bls12_381 as B
from oracle import hbbft_rules as RULES
from oracle import threshold_crypto as T

cb = pytest.importorskip("oracle.cbaseline", reason="oracle/c not built (make oracle)")

G1 = B.g1_compress(B.G1_GEN)


class OracleCtx:
    """Test double with the hbtc Context interface, computing with the C oracle."""

    def __init__(self):
        self.keysets = {}

    def keyset_load(self, pks):
        k = len(self.keysets) + 1
        self.keysets[k] = list(pks)
        return k, 0

    def verify_sig_shares(self, ks, H, counts, idx, sigs):
        out, pos = [], 0
        for k, c in enumerate(counts):
            for j in range(pos, pos + c):
                i = idx[j]
                r = cb.pairing_eq(self.keysets[ks][i], H[k], G1, sigs[j]) if i < len(self.keysets[ks]) else False
                out.append(N.ACCEPT if r else N.REJECT)
            pos += c
        return np.array(out, np.int32)

    def verify_sigs(self, pks, H, sigs):
        return np.array([N.ACCEPT if cb.pairing_eq(p, h, G1, s) else N.REJECT for p, h, s in zip(pks, H, sigs)], np.int32)

    def combine_sigs(self, counts, idx, sigs, t):
        return self._combine(2, counts, idx, sigs, t)

    def combine_dec(self, counts, idx, shares, t):
        out, _, st = self._combine(1, counts, idx, shares, t)
        return out, st

    def _combine(self, group, counts, idx, pts, t):
        out, par, st, pos = [], [], [], 0
        for c in counts:
            s, o = cb.combine(group, idx[pos:pos + c], pts[pos:pos + c], t)
            out.append(o)
            par.append(cb.sig_parity(o) if (s == 0 and group == 2) else 0)
            st.append({0: N.ACCEPT, 5: N.NOT_ENOUGH_SHARES, 6: N.DUPLICATE_ENTRY}.get(s, N.DECODE_ERR))
            pos += c
        return out, np.array(par, np.uint8), np.array(st, np.int32)

    def verify_dec_shares(self, ks, H, w, counts, idx, shares):
        out, pos = [], 0
        for k, c in enumerate(counts):
            for j in range(pos, pos + c):
                r = cb.pairing_eq(shares[j], H[k], self.keysets[ks][idx[j]], w[k])
                out.append(N.ACCEPT if r else N.REJECT)
            pos += c
        return np.array(out, np.int32)

    def verify_ciphertexts(self, us, H, ws):
        return np.array([N.ACCEPT if cb.pairing_eq(G1, w, u, h) else N.REJECT for u, h, w in zip(us, H, ws)], np.int32)


def keyset(rng, n):
    f = (n - 1) // 3
    coeffs = [rng.randrange(1, B.R) for _ in range(f + 1)]
    sks = [T.poly_evaluate(coeffs, i + 1) for i in range(n)]
    pks = [cb.g1_mul(G1, s) for s in sks]
    return sks, pks, cb.g1_mul(G1, coeffs[0])


def strip(steps):
    return [{"faults": s["faults"], "output": s["output"], "error": s["error"]} for s in steps]


def coin_scenario(rng, n, n_inst):
    ids = ["n%02d" % i for i in range(n)]
    sks, pks, mpk = keyset(rng, n)
    our = ids[rng.randrange(n)]
    g2 = B.g2_compress(B.G2_GEN)
    insts = {}
    for k in range(n_inst):
        H = cb.hash_g2(b"nonce %d" % k)
        shares = {ids[i]: cb.g2_mul(H, sks[i]) for i in range(n)}
        bad = rng.sample(ids, 2)
        for b in bad:
            shares[b] = cb.g2_mul(H, sks[0] + 1)
        events = [("msg", s, shares[s]) for s in rng.sample(ids, n)]
        events.append(("msg", "zz_unknown", shares[ids[1]]))
        events.append(("msg", ids[3], shares[ids[3]]))  # duplicate, maybe after termination
        rng.shuffle(events)
        events.insert(rng.randrange(len(events) + 1), ("input",))
        insts[k] = (H, shares[our] if our not in bad else cb.g2_mul(H, sks[ids.index(our)]), events)
    return ids, sks, pks, mpk, our, insts


def run_coin(ctx, rng, n=7, n_inst=3, n_flush=2, wrong_master=False):
    ids, sks, pks, mpk, our, insts = coin_scenario(rng, n, n_inst)
    f = (n - 1) // 3
    if wrong_master:  # every combine fails the master check: VerificationFailed, retried per share
        mpk = cb.g1_mul(G1, 12345)
    ks, _ = ctx.keyset_load(pks)
    ni = P.NetInfo(ids, our, ks, master_pk=mpk)
    ep = P.CoinEpoch(ctx, ni)
    for k, (H, own, _) in insts.items():
        ep.add(k, H, own)
    got = {k: [] for k in insts}
    for fi in range(n_flush):  # split every queue over several flushes
        for k, (H, own, events) in insts.items():
            lo, hi = len(events) * fi // n_flush, len(events) * (fi + 1) // n_flush
            for ev in events[lo:hi]:
                (ep.handle_input(k) if ev[0] == "input" else ep.handle_message(k, ev[1], ev[2]))
        for k, steps in ep.flush().items():
            got[k] += strip(steps)
    for k, (H, own, events) in insts.items():
        def verify(sender, share, H=H):
            return bool(cb.pairing_eq(pks[ids.index(sender)], H, G1, share))

        def comb(items):
            st, sig = cb.combine(2, [i for i, _ in items], [s for _, s in items], f + 1)
            if st:
                raise RuntimeError(st)
            return sig, bool(cb.sig_parity(sig))

        ref = RULES.Coin(ids, our, f, own, verify, comb, lambda sig, H=H: bool(cb.pairing_eq(mpk, H, G1, sig)))
        want = ref.run(events)
        assert got[k] == want, (k, events)
        if wrong_master:
            assert sum(s["error"] == "VerificationFailed" for s in want) >= 2
        else:
            assert any(s["output"] is not None for s in want)


def run_decryption(ctx, rng, n=7, n_ct=3, n_flush=2):
    ids = ["n%02d" % i for i in range(n)]
    sks, pks, mpk = keyset(rng, n)
    f = (n - 1) // 3
    our = ids[rng.randrange(n)]
    ks, _ = ctx.keyset_load(pks)
    ni = P.NetInfo(ids, our, ks, master_pk=mpk)
    ep = P.DecryptionEpoch(ctx, ni)
    cases = {}
    for k in range(n_ct):
        r = rng.randrange(1, B.R)
        u = cb.g1_mul(G1, r)
        v = bytes(rng.randrange(256) for _ in range(24))
        H = cb.hash_g1_g2(u, v)
        w = cb.g2_mul(H, r)
        w_bad = cb.g2_mul(H, r + 1)  # invalid ciphertext: set_ciphertext -> InvalidCiphertext
        if k == 2:
            w = w_bad
        shares = {ids[i]: cb.g1_mul(u, sks[i]) for i in range(n)}
        for b in rng.sample(ids, 2):
            shares[b] = cb.g1_mul(u, sks[0] + 5)
        events = [("msg", s, shares[s]) for s in rng.sample(ids, n)]
        events.append(("msg", "zz_unknown", shares[ids[0]]))
        events.append(("msg", ids[2], shares[ids[2]]))
        rng.shuffle(events)
        pos = rng.randrange(len(events) + 1)
        events.insert(pos, ("ct", (u, v, w, H)))
        if k == 1:  # an invalid ciphertext queued before the valid one: the valid one is accepted
            events.insert(rng.randrange(pos + 1), ("ct", (u, v, w_bad, H)))
        own = cb.g1_mul(u, sks[ids.index(our)])
        cases[k] = (own, events)
        ep.add(k, own)
    got = {k: [] for k in cases}
    for fi in range(n_flush):
        for k, (own, events) in cases.items():
            lo, hi = len(events) * fi // n_flush, len(events) * (fi + 1) // n_flush
            for ev in events[lo:hi]:
                if ev[0] == "ct":
                    ep.set_ciphertext(k, *ev[1])
                else:
                    ep.handle_message(k, ev[1], ev[2])
        for k, steps in ep.flush().items():
            got[k] += strip(steps)
    for k, (own, events) in cases.items():
        def verify(sender, share, ct):
            return bool(cb.pairing_eq(share, ct[3], pks[ids.index(sender)], ct[2]))

        def decrypt(items, ct):
            st, g = cb.combine(1, [i for i, _ in items], [s for _, s in items], f + 1)
            if st:
                raise RuntimeError(st)
            return g

        def ct_valid(ct):
            return bool(cb.pairing_eq(G1, ct[2], ct[0], ct[3]))

        ref = RULES.ThresholdDecryption(ids, our, f, own, verify, decrypt, ct_valid)
        want = ref.run(events)
        assert got[k] == want, (k, events)


@pytest.mark.parametrize("seed", [1, 2])
def test_coin_queue_matches_reference_rules_cpu(seed):
    run_coin(OracleCtx(), random.Random(seed))


@pytest.mark.parametrize("seed", [3, 4])
def test_decryption_queue_matches_reference_rules_cpu(seed):
    run_decryption(OracleCtx(), random.Random(seed))


@pytest.mark.parametrize("seed", [11, 12])
def test_coin_queue_failed_combine_retries_cpu(seed):
    """A deferred combine that fails keeps the shares and the input of earlier flushes
    (coin.rs:163-181 retries on every later share)."""
    run_coin(OracleCtx(), random.Random(seed), n_flush=3, wrong_master=True)


@pytest.fixture(scope="module")
def gctx():
    c = N.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [5, 6, 7])
def test_coin_queue_matches_reference_rules_gpu(gctx, seed):
    run_coin(gctx, random.Random(seed), n=10, n_inst=4, n_flush=3)


@pytest.mark.gpu
def test_coin_queue_failed_combine_retries_gpu(gctx):
    run_coin(gctx, random.Random(13), n=10, n_inst=3, n_flush=3, wrong_master=True)


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [8, 9])
def test_decryption_queue_matches_reference_rules_gpu(gctx, seed):
    run_decryption(gctx, random.Random(seed), n=10, n_ct=4, n_flush=3)
