"""Reliable Broadcast coding on the GPU — the host-side mirror of hbbft's src/broadcast/ coding
path over libhbtc.so (include/hbtc.h "Reliable Broadcast coding").

The reference codes one value at a time on the CPU: the proposer's ``send_shards``
(/root/reference/src/broadcast/broadcast.rs:150-211: length prefix, padding, ReedSolomon::encode,
MerkleTree::from_vec, one proof per node), every node's ``validate_proof`` of each Value / Echo
(:356-376, merkle.rs:82-102) and ``decode_from_shards`` (:461-493: reconstruct_shards, a new
Merkle tree, the root comparison, glue_shards).  A HoneyBadger epoch runs N broadcasts, so a
node checks N^2 Echo proofs and decodes N values per epoch; here each of those is ONE batched
call: ``validate_proofs`` (every queued proof), ``decode_batch`` (every instance ready to
decode: one reconstruction launch per presence pattern, one Merkle-tree launch), and
``send_shards`` / ``encode_batch`` for proposals.

Decisions and bytes equal the reference's (tests/test_broadcast.py checks them against
oracle/broadcast.py's restatement).  The Reed-Solomon matrices are reed-solomon-erasure 3.1's;
N <= 256 (ReedSolomon::new refuses more shards, so hbbft's Broadcast::new fails beyond it).
"""
import struct

import numpy as np

from . import _native as N


def shard_counts(num_nodes, num_faulty):
    """broadcast.rs:128-129: parity = 2f, data = N - 2f."""
    p = 2 * num_faulty
    return num_nodes - p, p


class Proof:
    """merkle.rs:72-77 Proof<Vec<u8>>."""

    __slots__ = ("value", "index", "digests", "root_hash")

    def __init__(self, value, index, digests, root_hash):
        self.value, self.index, self.digests, self.root_hash = bytes(value), index, list(digests), bytes(root_hash)


class MerkleTree:
    """merkle.rs:11-68 on the digests of one hbtc_merkle_trees row (level 0 first, root last)."""

    def __init__(self, values, digests):
        self.values = [bytes(v) for v in values]
        n = len(values)
        self.levels, pos, m = [], 0, n
        flat = [bytes(d) for d in digests]
        while m > 1:
            self.levels.append(flat[pos:pos + m])
            pos += m
            m = (m + 1) // 2
        self.root_hash = flat[-1]

    def proof(self, index):
        if index >= len(self.values):
            return None
        digests, i = [], index
        for lvl in self.levels:
            if (i ^ 1) < len(lvl):
                digests.append(lvl[i ^ 1])
            i //= 2
        return Proof(self.values[index], index, digests, self.root_hash)


def merkle_trees(ctx, values_per_inst):
    """MerkleTree::from_vec for several instances with equal leaf counts and lengths."""
    if not values_per_inst:
        return []
    n, ln = len(values_per_inst[0]), len(values_per_inst[0][0])
    buf = np.frombuffer(b"".join(bytes(v) for vs in values_per_inst for v in vs), np.uint8).copy()
    dig = ctx.merkle_trees(n, ln, buf)
    return [MerkleTree(vs, dig[i]) for i, vs in enumerate(values_per_inst)]


def padded_value(value, k, p):
    """send_shards' buffer (broadcast.rs:158-171): BE u32 length, the value, zeros to
    shard_len * (k + p)."""
    v = struct.pack(">I", len(value)) + bytes(value)
    shard_len = (len(v) + k - 1) // k
    return v + bytes(shard_len * (k + p) - len(v)), shard_len


def encode_batch(ctx, values, num_nodes, num_faulty):
    """send_shards for several proposals of equal shard length: uint8 array [n_inst, N, len]."""
    k, p = shard_counts(num_nodes, num_faulty)
    bufs = [padded_value(v, k, p) for v in values]
    shard_len = bufs[0][1]
    if any(sl != shard_len for _, sl in bufs):
        raise ValueError("encode_batch: proposals must share a shard length")
    a = np.frombuffer(b"".join(b for b, _ in bufs), np.uint8).copy()
    if p:
        ctx.rs_encode(k, p, shard_len, a)
    return a.reshape(len(values), k + p, shard_len)


def send_shards(ctx, value, num_nodes, num_faulty):
    """Broadcast::send_shards: (shards, tree, proofs) — proof i goes to node i."""
    sh = encode_batch(ctx, [value], num_nodes, num_faulty)[0]
    shards = [bytes(s) for s in sh]
    tree = merkle_trees(ctx, [shards])[0]
    return shards, tree, [tree.proof(i) for i in range(num_nodes)]


def validate_proofs(ctx, proofs, num_nodes, expected_index=None):
    """validate_proof (broadcast.rs:358-376) of many proofs in one call: Proof::validate(N) and,
    with expected_index, the sender's node index == proof.index.  Returns a bool array."""
    if not proofs:
        return np.zeros(0, bool)
    if not 0 < num_nodes < 1 << 31:
        raise ValueError("validate_proofs: num_nodes out of range")
    # The wire index is a usize (u64).  The device walk takes a u32: an index of 2^32 or more
    # walks exactly like 2^32 - 1 (index ^ 1 >= the level size on every level while the node
    # count is below 2^31, so no digest is consumed), so one Byzantine Echo with a huge index
    # gets its own verdict (valid iff it has no digests and its leaf hash is the root, as in the
    # reference) instead of failing the whole batch.
    ix = [p.index if 0 <= p.index < 1 << 32 else (1 << 32) - 1 for p in proofs]
    st = ctx.merkle_validate(num_nodes, [p.value for p in proofs], ix,
                             [p.digests for p in proofs], [p.root_hash for p in proofs])
    ok = st == N.ACCEPT
    if expected_index is not None:
        ok &= np.asarray([p.index for p in proofs]) == np.asarray(expected_index)
    return ok


def glue_shards(values, k):
    """broadcast.rs:498-508."""
    data = b"".join(bytes(v) for v in values[:k])
    if len(data) < 4:
        return None
    return data[4:4 + struct.unpack(">I", data[:4])[0]]


# SHA3-256 of the empty string (FIPS 202): the digest of an empty leaf
_SHA3_EMPTY = bytes.fromhex("a7ffc6f8bf1ed76651c14756a061d662f580ff4de43b49fa82d80a4b80f8434a")


def _sha3_many(ctx, blobs):
    """SHA3-256 of each byte string on the GPU, one hbtc_merkle_trees call per distinct length
    (the root of a one-leaf tree is that leaf's digest)."""
    out, by_len = [None] * len(blobs), {}
    for i, b in enumerate(blobs):
        by_len.setdefault(len(b), []).append(i)
    for ln, ids in by_len.items():
        if ln == 0:
            for i in ids:
                out[i] = _SHA3_EMPTY
            continue
        dig = ctx.merkle_trees(1, ln, np.frombuffer(b"".join(blobs[i] for i in ids), np.uint8).copy())
        for r, i in enumerate(ids):
            out[i] = bytes(dig[r, -1])
    return out


def _ragged_root(ctx, leaves):
    """MerkleTree::from_vec(leaves).root_hash() for leaves of any lengths (merkle.rs:19-32: the
    odd digest of a level is carried up unhashed)."""
    cur = _sha3_many(ctx, leaves)
    while len(cur) > 1:
        h = _sha3_many(ctx, [cur[i] + cur[i + 1] for i in range(0, len(cur) - 1, 2)])
        cur = [h[j // 2] if j + 1 < len(cur) else cur[j] for j in range(0, len(cur), 2)]
    return cur[0]


def decode_batch(ctx, leaf_values_per_inst, root_hashes, num_faulty):
    """decode_from_shards (broadcast.rs:461-493) for several instances of one network (every
    leaf list has N entries, bytes or None).  Reed-Solomon instances need one shard length
    (IncorrectShardSize otherwise); the trivial coding (no parity shards) takes any lengths.
    Returns the decoded value or None per instance, as the reference."""
    out = [None] * len(leaf_values_per_inst)
    if not leaf_values_per_inst:
        return out
    n = len(leaf_values_per_inst[0])
    k, p = shard_counts(n, num_faulty)
    # instances grouped by shard length (one reconstruction call each)
    by_len = {}
    for i, lv in enumerate(leaf_values_per_inst):
        lens = {len(v) for v in lv if v is not None}
        if p == 0 and all(v is not None for v in lv) and (len(lens) != 1 or 0 in lens):
            # Coding::Trivial checks presence only (broadcast.rs:449-455): the tree is built over
            # the leaves as they are, whatever their lengths
            leaves = [bytes(v) for v in lv]
            if _ragged_root(ctx, leaves) == bytes(root_hashes[i]):
                out[i] = glue_shards(leaves, k)
            continue
        if len(lens) != 1 or 0 in lens:  # IncorrectShardSize / nothing present / empty shards
            continue
        by_len.setdefault(lens.pop(), []).append(i)
    for ln, insts in by_len.items():
        buf = np.zeros((len(insts), n, ln), np.uint8)
        present = np.zeros((len(insts), n), np.uint8)
        for r, i in enumerate(insts):
            for j, v in enumerate(leaf_values_per_inst[i]):
                if v is not None:
                    buf[r, j] = np.frombuffer(v, np.uint8)
                    present[r, j] = 1
        if p:
            _, st = ctx.rs_reconstruct(k, p, ln, buf.reshape(-1), present.reshape(-1))
            ok = st == N.ACCEPT
        else:  # the trivial coding: every shard must be present
            ok = present.all(axis=1)
        good = [r for r in range(len(insts)) if ok[r]]
        if not good:
            continue
        dig = ctx.merkle_trees(n, ln, buf[good].reshape(-1))
        for gi, r in enumerate(good):
            if bytes(dig[gi, -1]) == bytes(root_hashes[insts[r]]):
                out[insts[r]] = glue_shards([bytes(buf[r, j]) for j in range(k)], k)
    return out
