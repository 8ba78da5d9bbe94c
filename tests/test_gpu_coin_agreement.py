"""tests/coin.rs:27-131 restated through the Coin batch queue (hbbft_amd/protocol.py CoinEpoch).

A network of good nodes, silent faulty nodes and an observer runs many Coin instances (one
nonce each, "My very unique nonce {id:x}:{i}" as in coin.rs:106).  Every good node inputs,
multicasts its SignatureShare (sk_i * hash_g2(nonce)), and every node (good nodes and the
observer) receives the other good nodes' shares in its own random order, over several flushes.
As in test_coin (coin.rs:27-51): every good node terminates with exactly one output, all good
nodes output the same value, the observer outputs it too; and over the instances both values
occur as often as check_coin_distribution (coin.rs:58-72) requires.  Network sizes follow
test_coin_different_sizes (coin.rs:74-119): 1, then steps of 3..6.
"""
import math
import random

import pytest

from hbbft_amd import _native as N
from hbbft_amd import protocol as P

pytestmark = pytest.mark.gpu
R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
G1 = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
OBSERVER = 10 ** 6


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    c.set_verify_mode(N.MODE_RLC)
    yield c
    c.close()


def _check_coin_distribution(num_samples, count_true, count_false):  # coin.rs:58-72
    max_gain = math.log2(400.0)
    gain = min(math.log2(num_samples), max_gain)
    min_throws = int(num_samples * gain * (0.4 / max_gain))
    assert count_true > min_throws and count_false > min_throws, (count_true, count_false, min_throws)


def _run(ctx, rng, size, num_samples, flushes):
    faulty = (size - 1) // 3
    good = size - faulty
    ids = list(range(size))
    coeffs = [rng.randrange(1, R) for _ in range(faulty + 1)]
    sks = [sum(c * pow(i + 1, j, R) for j, c in enumerate(coeffs)) % R for i in ids]
    pk, _ = ctx.g1_mul(G1, sks)
    mpk, _ = ctx.g1_mul(G1, [coeffs[0]])
    ks, bad = ctx.keyset_load(pk)
    assert bad == 0
    unique_id = rng.getrandbits(64)
    nonces = [("My very unique nonce %x:%d" % (unique_id, i)).encode() for i in range(num_samples)]
    Hs = N.hash_g2_batch(nonces)
    shares = {}
    for i in range(good):  # faulty nodes ids good..size-1 stay silent
        sig, st = ctx.g2_mul(Hs, [sks[i]] * num_samples)
        assert not st.any()
        shares[i] = [bytes(sig[96 * k:96 * k + 96]) for k in range(num_samples)]
    outputs = {}
    for node in list(range(good)) + [OBSERVER]:
        ep = P.CoinEpoch(ctx, P.NetInfo(ids, node, ks, master_pk=bytes(mpk)))
        for k in range(num_samples):
            ep.add(k, Hs[k], shares[node][k] if node in shares else None)
            ep.handle_input(k)
        msgs = [(k, s) for k in range(num_samples) for s in range(good) if s != node]
        rng.shuffle(msgs)
        outs = {k: [] for k in range(num_samples)}
        cuts = sorted(rng.sample(range(1, len(msgs)), min(flushes - 1, max(0, len(msgs) - 1)))) \
            if msgs else []
        bounds = [0] + cuts + [len(msgs)]
        first = True
        for a, b in zip(bounds, bounds[1:]):
            for k, s in msgs[a:b]:
                ep.handle_message(k, s, shares[s][k])
            if first or b > a:
                res = ep.flush()
                first = False
                for k, steps in res.items():
                    for st in steps:
                        assert st["error"] is None and not st["faults"], st
                        if st["output"] is not None:
                            outs[k].append(st["output"])
        outputs[node] = outs
    ctx.keyset_free(ks)
    values = []
    for k in range(num_samples):
        ref = outputs[0][k]
        assert len(ref) == 1, (size, k, ref)
        for node in range(good):
            assert outputs[node][k] == ref
        assert outputs[OBSERVER][k] == ref
        values.append(ref[0])
    return values


@pytest.mark.timeout(300)
def test_coin_network_agreement_and_distribution(ctx):
    rng = random.Random(2718)
    num_samples = 200
    sizes, last = [1], 1
    for _ in range(int(math.log2(400.0) - math.log2(num_samples))):
        last += rng.randrange(3, 7)
        sizes.append(last)
    sizes += [10, 16]
    for size in sizes:
        vals = _run(ctx, rng, size, num_samples, flushes=3)
        _check_coin_distribution(num_samples, sum(vals), num_samples - sum(vals))
