"""Host hash_g2 / hash_g1_g2 (hbtc_hash_g2, hbtc_hash_g1_g2; include/hbtc.h) against the oracle's
restatement of threshold_crypto's crate-internal hashes (oracle/threshold_crypto.py:
hash_g2 / hash_g1_g2 over oracle/rand04.py's ChaChaRng).  Host code: runs without a GPU.

Both sides restate the same published algorithm [EXT-UNVERIFIED]; agreement pins the C++
product against the oracle, not against real threshold_crypto bytes (parity unpinned,
DESIGN.md §2).  SHA3-256 is pinned against hashlib (FIPS 202)."""
import hashlib
import random

import pytest

from hbbft_amd import _native as N
from oracle import bls12_381 as B
from oracle import threshold_crypto as TC


@pytest.mark.parametrize("n", [0, 1, 64, 135, 136, 137, 300, 1000])
def test_sha3_256_matches_hashlib(n):
    msg = bytes(random.Random(n).randrange(256) for _ in range(n))
    assert N.sha3_256(msg) == hashlib.sha3_256(msg).digest()


COIN_NONCE = (b"Nonce for Honey Badger [173, 84, 2, 11, 0, 0, 9, 254, 1, 18, 200, 57, 43, 9, "
              b"4, 77, 190, 91, 12, 0, 1, 2, 3]@3:2:7")


@pytest.mark.parametrize("msg", [b"", b"hbbft", COIN_NONCE, bytes(range(200))])
def test_hash_g2_matches_oracle(msg):
    got = N.hash_g2(msg)
    want = B.g2_compress(TC.hash_g2(msg))
    assert got == want
    # the result is a valid prime-order G2 point (decompress checks the subgroup)
    assert B.g2_decompress(got) is not None


@pytest.mark.parametrize("vlen", [0, 64, 65, 200])
def test_hash_g1_g2_matches_oracle(vlen):
    rng = random.Random(vlen)
    u = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
    v = bytes(rng.randrange(256) for _ in range(vlen))
    got = N.hash_g1_g2(B.g1_compress(u), v)
    assert got == B.g2_compress(TC.hash_g1_g2(u, v))


def test_batches_match_single_calls():
    rng = random.Random(9)
    msgs = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 150))) for _ in range(12)]
    assert N.hash_g2_batch(msgs) == [N.hash_g2(m) for m in msgs]
    us = [B.g1_compress(B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))) for _ in msgs]
    assert N.hash_g1_g2_batch(us, msgs) == [N.hash_g1_g2(u, m) for u, m in zip(us, msgs)]
    assert N.hash_g2_batch([]) == []


@pytest.mark.parametrize("length", [0, 1, 40, 64, 4097])
def test_hash_bytes_matches_oracle(length):
    rng = random.Random(length + 5)
    g = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
    assert N.hash_bytes(B.g1_compress(g), length) == TC.hash_bytes(g, length)


def test_xor_hash_bytes_batch_roundtrip():
    """The encrypt / decrypt pad: msg XOR pad XOR pad == msg, and each pad is hash_bytes(g)."""
    rng = random.Random(77)
    gs = [B.g1_compress(B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))) for _ in range(9)]
    msgs = [bytes(rng.randrange(256) for _ in range(rng.randrange(0, 300))) for _ in gs]
    enc = N.xor_hash_bytes_batch(gs, msgs)
    for g, m, e in zip(gs, msgs, enc):
        assert bytes(a ^ b for a, b in zip(e, m)) == N.hash_bytes(g, len(m))
    assert N.xor_hash_bytes_batch(gs, enc) == msgs
