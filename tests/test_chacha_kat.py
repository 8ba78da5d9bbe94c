"""ChaCha20 known-answer tests for rand 0.4's ChaChaRng — the keystream under threshold_crypto's
hash_g2 / hash_g1_g2 / hash_bytes (rand = "0.4.2", /root/reference/Cargo.toml:28; the crate is
not vendored).

The vectors are rand 0.4's own `test_rng_true_values` (src/prng/chacha.rs): the all-zero seed's
first two blocks — which are also the ChaCha20 block function's published zero-key, zero-nonce
vectors for counters 0 and 1 (RFC 7539 A.1 #1 / #2, read as little-endian words) — and, for the
seed words 0..7, the i-th word of the i-th block for i < 16 (key-word layout and the block
counter across 17 blocks).  They pin the keystream of oracle/rand04.py, of the product's host
hashes (hbtc_chacha04_words) and of the GPU candidate kernel (hbtc_chacha04_words_gpu, gpu
marker).  Still unpinned: how threshold_crypto turns the SHA3 digest into the
seed words, next_u64's word order, and G2::rand's rejection details."""
import numpy as np
import pytest

from hbbft_amd import _native as N
from oracle.rand04 import ChaChaRng

ZERO_BLOCK0 = [0xade0b876, 0x903df1a0, 0xe56a5d40, 0x28bd8653, 0xb819d2bd, 0x1aed8da0,
               0xccef36a8, 0xc70d778b, 0x7c5941da, 0x8d485751, 0x3fe02477, 0x374ad8b8,
               0xf4b8436a, 0x1ca11815, 0x69b687c3, 0x8665eeb2]
ZERO_BLOCK1 = [0xbee7079f, 0x7a385155, 0x7c97ba98, 0x0d082d73, 0xa0290fcb, 0x6965e348,
               0x3e53c612, 0xed7aee32, 0x7621b729, 0x434ee69c, 0xb03371d5, 0xd539d874,
               0x281fed31, 0x45fb0a51, 0x1f0ae1ac, 0x6f4d794b]
SEQ_DIAGONAL = [0xf225c81a, 0x6ab1be57, 0x04d42951, 0x70858036, 0x49884684, 0x64efec72,
                0x4be2d186, 0x3615b384, 0x11cfa18e, 0xd3c50049, 0x75c775f6, 0x434c6530,
                0x2c5bad8f, 0x898881dc, 0x5f1c86d9, 0xc1f8e7f4]
# RFC 7539 A.1 test vector #1 (key 0, nonce 0, counter 0), keystream bytes
RFC_ZERO_BYTES = bytes.fromhex(
    "76b8e0ada0f13d90405d6ae55386bd28bdd219b8a08ded1aa836efcc8b770dc7"
    "da41597c5157488d7724e03fb8d84a376a43b8f41518a11cc387b669b2ee6586")


def _diagonal(words):
    return [int(words[17 * i]) for i in range(16)]


def _check(zero32, seq272):
    assert [int(x) for x in zero32[:16]] == ZERO_BLOCK0
    assert [int(x) for x in zero32[16:32]] == ZERO_BLOCK1
    assert np.asarray(zero32[:16], "<u4").tobytes() == RFC_ZERO_BYTES
    assert _diagonal(seq272) == SEQ_DIAGONAL


def test_oracle_rand04_known_answers():
    r = ChaChaRng([0] * 8)
    zero = [r.next_u32() for _ in range(32)]
    r = ChaChaRng(list(range(8)))
    seq = [r.next_u32() for _ in range(17 * 16)]
    _check(zero, seq)


def test_host_hash_chacha_known_answers():
    _check(N.chacha04_words([0] * 8, 32), N.chacha04_words(list(range(8)), 17 * 16))


def test_host_chacha_matches_oracle_for_digest_seeds():
    """Past the KATs: the host stream equals the oracle's on seeds of the hashes' shape."""
    rng = np.random.default_rng(5)
    for _ in range(4):
        seed = [int(x) for x in rng.integers(0, 2 ** 32, 8, dtype=np.uint64)]
        r = ChaChaRng(seed)
        assert [int(x) for x in N.chacha04_words(seed, 100)] == [r.next_u32() for _ in range(100)]


@pytest.mark.gpu
def test_gpu_hash_chacha_known_answers():
    ctx = N.Context(0)
    try:
        _check(ctx.chacha04_words([0] * 8, 32), ctx.chacha04_words(list(range(8)), 17 * 16))
    finally:
        ctx.close()
