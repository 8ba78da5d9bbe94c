"""hash_g2 / hash_g1_g2 with the full-cofactor multiplication on the GPU
(hbtc_hash_g2_batch_gpu / hbtc_hash_g1_g2_batch_gpu) against the oracle restatement
(oracle/threshold_crypto.py) and the host path (tests/test_hash.py pins that one).  Bar:
identical bytes.  Parity against real threshold_crypto bytes: unpinned."""
import random
import time

import pytest

from hbbft_amd import _native as N
from oracle import bls12_381 as B
from oracle import threshold_crypto as TC

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    yield c
    c.close()


def test_gpu_hash_g2_matches_oracle_and_host(ctx):
    rng = random.Random(3)
    msgs = [b"", b"hbbft"] + [bytes(rng.randrange(256) for _ in range(rng.randrange(1, 120)))
                              for _ in range(70)]
    msgs += [bytes(rng.randrange(256) for _ in range(L)) for L in (135, 136, 137, 271, 272, 500)]
    got = ctx.hash_g2_batch(msgs)
    assert got == N.hash_g2_batch(msgs)
    for m in msgs[:3]:
        assert got[msgs.index(m)] == B.g2_compress(TC.hash_g2(m))


def test_gpu_hash_g1_g2_matches_oracle(ctx):
    rng = random.Random(4)
    us = [B.g1_mul(B.G1_GEN, rng.randrange(1, B.R)) for _ in range(3)]
    vs = [bytes(rng.randrange(256) for _ in range(n)) for n in (0, 64, 200)]
    got = ctx.hash_g1_g2_batch([B.g1_compress(u) for u in us], vs)
    assert got == [B.g2_compress(TC.hash_g1_g2(u, v)) for u, v in zip(us, vs)]


def test_gpu_hash_epoch_batch_throughput(ctx):
    """C3's 1000 per-ciphertext hashes: GPU batch equals the host batch; times printed."""
    rng = random.Random(5)
    us = [bytes([0x97]) + bytes(rng.randrange(256) for _ in range(47)) for _ in range(1000)]
    vs = [bytes(rng.randrange(256) for _ in range(64)) for _ in range(1000)]
    ctx.hash_g1_g2_batch(us[:64], vs[:64])  # warm
    t0 = time.perf_counter()
    got = ctx.hash_g1_g2_batch(us, vs)
    t1 = time.perf_counter()
    want = N.hash_g1_g2_batch(us, vs)
    t2 = time.perf_counter()
    print("1000 hash_g1_g2: GPU cofactor %.1f ms, host-only %.1f ms" % ((t1 - t0) * 1e3, (t2 - t1) * 1e3))
    assert got == want
