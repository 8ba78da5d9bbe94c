"""Reliable Broadcast coding (src/broadcast/): the oracle restatement against the reference's own
tests (merkle.rs:146-160, tests/broadcast.rs scenarios) and properties on CPU; the GPU path
(hbbft_amd/broadcast.py over hbtc_rs_* / hbtc_merkle_*) against the oracle byte for byte under
-m gpu.  Parity of the Reed-Solomon parity BYTES with reed-solomon-erasure 3.1 rests on the
crate's published construction (oracle/broadcast.py); everything else (Merkle digests =
FIPS 202 SHA3-256, decode results) is pinned by hashlib and by the round trips."""
import hashlib
import random

import numpy as np
import pytest

from oracle import broadcast as B


# ------------------------------------------------------------------ CPU: the oracle
def test_reference_merkle_test():
    """merkle.rs:150-160 test_merkle: every proof of trees of 4, 7, 8, 9, 17 one-byte values
    validates, and there is no proof past the end."""
    for n in (4, 7, 8, 9, 17):
        vals = [bytes([i]) for i in range(n)]
        levels, root = B.merkle_levels(vals)
        for i in range(n):
            assert B.proof_validate(B.merkle_proof(levels, root, vals, i), n)
        assert B.merkle_proof(levels, root, vals, n) is None


def test_merkle_known_answer_and_tampering():
    vals = [b"a", b"b", b"c"]
    levels, root = B.merkle_levels(vals)
    h = lambda x: hashlib.sha3_256(x).digest()
    assert root == h(h(h(b"a") + h(b"b")) + h(b"c"))  # the odd digest is carried up unhashed
    pr = B.merkle_proof(levels, root, vals, 2)
    assert pr[2] == [h(h(b"a") + h(b"b"))]
    v, i, d, r = B.merkle_proof(levels, root, vals, 1)
    assert not B.proof_validate((b"x", i, d, r), 3)          # wrong value
    assert not B.proof_validate((v, 0, d, r), 3)             # wrong index
    assert not B.proof_validate((v, i, d[:-1], r), 3)        # too few levels
    assert not B.proof_validate((v, i, d + [d[0]], r), 3)    # too many levels
    assert not B.proof_validate((v, i, d, bytes(32)), 3)     # wrong root


def test_rs_matrix_systematic_and_mds():
    k, p = 5, 8
    m = B.build_matrix(k, k + p)
    assert all(m[i][j] == (i == j) for i in range(k) for j in range(k))
    rng = random.Random(3)
    for _ in range(20):  # any k rows are invertible (MDS)
        B.mat_inv([m[i] for i in sorted(rng.sample(range(k + p), k))])
    with pytest.raises(B.CodingError):
        B.build_matrix(100, 257)


@pytest.mark.parametrize("n", [1, 2, 3, 4, 5, 7, 16, 31, 64])
def test_send_decode_round_trip(n):
    """tests/broadcast.rs: a value proposed to n nodes is decoded from any N - 2f shards (the
    first delivered, random subsets), equal to the proposal; a tampered shard is caught by the
    root check."""
    rng = random.Random(n)
    f = (n - 1) // 3
    k, p = B.shard_counts(n, f)
    for val in (b"Foo", b"RandomFoo", b" " * 32, bytes(rng.randrange(256) for _ in range(300))):
        shards, levels, root, proofs = B.send_shards(val, n, f)
        assert all(B.proof_validate(pr, n) for pr in proofs)
        keep = sorted(rng.sample(range(n), k))
        lv = [s if i in keep else None for i, s in enumerate(shards)]
        assert B.decode_from_shards(lv, f, root) == val
        if p:
            bad = list(lv)
            j = keep[0]
            bad[j] = bytes([bad[j][0] ^ 1]) + bad[j][1:]
            assert B.decode_from_shards(bad, f, root) is None
            too_few = [s if i in keep[:-1] else None for i, s in enumerate(shards)]
            assert B.decode_from_shards(too_few, f, root) is None


def test_equal_leaves_scenario():
    """tests/broadcast.rs:145-153 test_8_broadcast_equal_leaves_silent: 32 spaces over 8 nodes
    (f = (8 - 1) / 3 = 2 as NetworkInfo computes it: 4 data + 4 parity shards of 9 bytes)."""
    shards, levels, root, proofs = B.send_shards(b" " * 32, 8, 2)
    assert len(shards) == 8 and all(len(s) == 9 for s in shards)
    assert shards[1:4] == [b" " * 9] * 3  # equal data leaves
    for keep in ([0, 1, 2, 3], [4, 5, 6, 7], [1, 3, 5, 7]):
        lv = [s if i in keep else None for i, s in enumerate(shards)]
        assert B.decode_from_shards(lv, 2, root) == b" " * 32


# ------------------------------------------------------------------ GPU: the product path
@pytest.fixture(scope="module")
def ctx():
    from hbbft_amd import _native as N
    c = N.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 7, 10, 64, 100, 256])
def test_gpu_send_shards_equal_oracle(ctx, n):
    from hbbft_amd import broadcast as G
    rng = random.Random(100 + n)
    f = (n - 1) // 3
    for size in (0, 3, 1000, 4097):
        val = bytes(rng.randrange(256) for _ in range(size))
        shards, tree, proofs = G.send_shards(ctx, val, n, f)
        o_shards, o_levels, o_root, o_proofs = B.send_shards(val, n, f)
        assert shards == o_shards
        assert tree.root_hash == o_root
        assert [(p.value, p.index, p.digests, p.root_hash) for p in proofs] == [
            (v, i, d, r) for v, i, d, r in o_proofs]


@pytest.mark.gpu
def test_gpu_validate_proofs_equal_oracle(ctx):
    """N = 31: every Echo proof of 3 instances plus tampered ones (value, index, digest count,
    a digest, the root); the GPU verdicts equal Proof::validate's."""
    from hbbft_amd import broadcast as G
    rng = random.Random(7)
    n, f = 31, 10
    proofs, exp = [], []
    for inst in range(3):
        val = bytes(rng.randrange(256) for _ in range(rng.randrange(1, 500)))
        _, _, root, ps = B.send_shards(val, n, f)
        for v, i, d, r in ps:
            variants = [(v, i, d, r)]
            if i % 5 == 0:
                variants += [(v[:-1] + bytes([v[-1] ^ 1]), i, d, r), (v, (i + 1) % n, d, r),
                             (v, i, d[:-1], r), (v, i, d + [r], r), (v, i, d, bytes(32)),
                             (v, i, [bytes(32)] + d[1:], r)]
            for var in variants:
                proofs.append(G.Proof(*var))
                exp.append(B.proof_validate(var, n))
    got = G.validate_proofs(ctx, proofs, n)
    assert list(got) == exp and sum(exp) == 3 * n


@pytest.mark.gpu
@pytest.mark.parametrize("n", [4, 16, 100, 256])
def test_gpu_decode_batch_equal_oracle(ctx, n):
    """decode_from_shards of many instances with different presence patterns (first k, random,
    all present, too few, a tampered shard) equals the restatement."""
    from hbbft_amd import broadcast as G
    rng = random.Random(n)
    f = (n - 1) // 3
    k, p = B.shard_counts(n, f)
    leafs, roots, exp = [], [], []
    for inst in range(12):
        val = bytes(rng.randrange(256) for _ in range(rng.choice([5, 200, 3000])))
        shards, _, root, _ = B.send_shards(val, n, f)
        kind = inst % 6
        if kind == 0:
            keep = set(range(n))
        elif kind == 1:
            keep = set(range(n - k, n))       # parity only (no data shard)
        elif kind == 2:
            keep = set(rng.sample(range(n), k))
        elif kind == 3:
            keep = set(rng.sample(range(n), max(k - 1, 0)))  # too few (p > 0)
        else:
            keep = set(rng.sample(range(n), min(n, k + rng.randrange(0, p + 1))))
        lv = [s if i in keep else None for i, s in enumerate(shards)]
        if kind == 5 and p:
            j = sorted(keep)[-1]
            lv[j] = bytes([lv[j][0] ^ 0x40]) + lv[j][1:]
        leafs.append(lv)
        roots.append(root)
        exp.append(B.decode_from_shards(lv, f, root))
    got = G.decode_batch(ctx, leafs, roots, f)
    assert got == exp
    assert any(v is not None for v in exp)


@pytest.mark.gpu
def test_gpu_validate_proofs_oversized_index(ctx):
    """A wire index (usize) of 2^32 or more: Proof::validate walks no level with it, so it is
    valid iff it has no digests and its leaf hash is the root; the other proofs of the batch
    keep their own verdicts, and the expected-index check rejects it."""
    from hbbft_amd import broadcast as G
    n, f = 7, 2
    _, _, root, ps = B.send_shards(b"oversized", n, f)
    v0 = ps[0][0]
    lone = hashlib.sha3_256(v0).digest()
    var = [ps[3], (v0, 1 << 40, [], lone), (v0, 1 << 32, ps[0][2], root), (v0, (1 << 64) - 1, [], lone),
           (v0, (1 << 32) - 1, [], lone), ps[5]]
    exp = [B.proof_validate(x, n) for x in var]
    assert exp == [True, True, False, True, True, True]
    got = G.validate_proofs(ctx, [G.Proof(*x) for x in var], n)
    assert list(got) == exp
    got = G.validate_proofs(ctx, [G.Proof(*x) for x in var], n, expected_index=[3, 1, 0, 0, 0, 5])
    assert list(got) == [True, False, False, False, False, True]


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpu_trivial_coding_ragged_leaves(ctx, n):
    """Coding::Trivial (no parity shards, N <= 3) checks presence only: leaves of different
    lengths (and empty ones) are hashed as they are, and the value glued if the root matches."""
    from hbbft_amd import broadcast as G
    rng = random.Random(50 + n)
    leafs, roots, exp = [], [], []
    for inst in range(8):
        lv = [bytes(rng.randrange(256) for _ in range(rng.choice([0, 1, 3, 4, 9, 40])))
              for _ in range(n)]
        if inst % 2 == 0:  # a prefix that glues to a value
            lv[0] = (3).to_bytes(4, "big") + b"abc" + lv[0]
        root = B.merkle_levels(lv)[1] if inst != 5 else bytes(32)
        if inst == 7 and n > 1:
            lv[1] = None  # missing: TooFewShardsPresent
        leafs.append(lv)
        roots.append(root)
        exp.append(B.decode_from_shards(lv, 0, root))
    assert G.decode_batch(ctx, leafs, roots, 0) == exp
    assert any(v is not None for v in exp)


@pytest.mark.gpu
def test_gpu_rs_counts_refused(ctx):
    from hbbft_amd import _native as N
    with pytest.raises(N.HbtcError):
        ctx.rs_encode(200, 100, 4, np.zeros(300 * 4, np.uint8))


@pytest.mark.gpu
@pytest.mark.parametrize("k,p,ln", [(250, 6, 37), (254, 2, 8), (3, 253, 5), (86, 170, 1)])
def test_gpu_rs_wide_codes_equal_oracle(ctx, k, p, ln):
    """Codes at the GF(2^8) limit (k + p = 256): k up to 254 input rows per output row (the
    kernel's LDS table block then exceeds 64 KB), odd shard lengths, one-byte shards; encode and
    reconstruct equal the restatement."""
    rng = np.random.default_rng(k * 1000 + p)
    n_inst = 3
    data = rng.integers(0, 256, (n_inst, k + p, ln), dtype=np.uint8)
    enc = ctx.rs_encode(k, p, ln, data.copy()).reshape(n_inst, k + p, ln)
    for i in range(n_inst):
        exp = B.rs_encode([bytes(r) for r in data[i]], k, p)
        assert [bytes(r) for r in enc[i]] == exp
    present = np.ones((n_inst, k + p), np.uint8)
    for i in range(n_inst):
        present[i, rng.choice(k + p, p, replace=False)] = 0
    recv = enc.copy()
    recv[present == 0] = 0
    out, st = ctx.rs_reconstruct(k, p, ln, recv.reshape(-1), present.reshape(-1))
    from hbbft_amd import _native as N
    assert (st == N.ACCEPT).all()
    assert np.array_equal(out.reshape(n_inst, k + p, ln), enc)
