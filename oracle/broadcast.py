"""CPU restatement of hbbft's Reliable Broadcast coding path (TEST INFRASTRUCTURE: only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg use it, as the checker; the product path
is hbbft_amd/broadcast.py over libhbtc.so).

What it restates:
  * reed-solomon-erasure 3.1.x (/root/reference/Cargo.toml:30; NOT vendored under
    /root/reference): GF(2^8) with the generating polynomial x^8 + x^4 + x^3 + x^2 + 1 (0x11D,
    the crate's `GENERATING_POLYNOMIAL = 29`) and generator 2; `galois_8::exp(a, n)` (a^n, with
    exp(a, 0) = 1 and exp(0, n > 0) = 0); the encoding matrix `build_matrix(k, n)` =
    vandermonde(n, k) * inverse(top k x k of it) (systematic: the top k rows are the identity);
    `encode` (parity row r = sum_j M[k + r][j] * data[j]); `reconstruct_shards` (the first k
    present shards in index order, the inverse of their rows of M, the missing data shards,
    then the missing parity shards re-encoded from the data).  The crate's published algorithm
    (Backblaze JavaReedSolomon); the parity BYTES are pinned here only by the crate's published
    construction, the round trips by the MDS property (see tests/test_broadcast.py).
  * /root/reference/src/broadcast/merkle.rs:19-32 MerkleTree::from_vec (leaf = sha3_256(value),
    a level's odd last digest is carried up unhashed), :35-52 proof, :82-102 Proof::validate,
    :127-144 hash_chunk / hash_pair / hash (tiny-keccak 1.4 sha3_256 = FIPS 202 SHA3-256 =
    hashlib.sha3_256).
  * /root/reference/src/broadcast/broadcast.rs:150-211 send_shards (u32 big-endian length
    prefix, shard_len = ceil(len / k), zero padding, parity, Merkle tree, proofs),
    :461-493 decode_from_shards, :498-508 glue_shards, :126-130 the shard counts
    (parity = 2f, data = N - 2f), :404-414 Coding (no parity shards: the trivial coding).
"""
import hashlib
import struct

import numpy as np

GF_POLY = 0x11D

_EXP = np.zeros(512, np.uint8)
_LOG = np.zeros(256, np.int32)
_x = 1
for _i in range(255):
    _EXP[_i] = _x
    _LOG[_x] = _i
    _x <<= 1
    if _x & 0x100:
        _x ^= GF_POLY
_EXP[255:510] = _EXP[0:255]
GF_EXP = _EXP
GF_LOG = _LOG


def gf_mul(a, b):
    if a == 0 or b == 0:
        return 0
    return int(_EXP[_LOG[a] + _LOG[b]])


def gf_exp(a, n):
    """galois_8::exp."""
    if n == 0:
        return 1
    if a == 0:
        return 0
    return int(_EXP[(int(_LOG[a]) * n) % 255])


def gf_inv(a):
    assert a != 0
    return int(_EXP[(255 - _LOG[a]) % 255])


# full multiplication table: MUL[a, b] = a * b in GF(2^8)
MUL = np.zeros((256, 256), np.uint8)
for _a in range(1, 256):
    MUL[_a, 1:] = _EXP[_LOG[_a] + _LOG[np.arange(1, 256)]]


def mat_mul(a, b):
    """GF(2^8) matrix product (lists of rows of ints)."""
    n, k, m = len(a), len(b), len(b[0])
    out = []
    for i in range(n):
        row = np.zeros(m, np.uint8)
        for j in range(k):
            if a[i][j]:
                row ^= MUL[a[i][j], np.asarray(b[j], np.uint8)]
        out.append([int(v) for v in row])
    return out


def mat_inv(m):
    """Gauss-Jordan inverse over GF(2^8); ValueError when singular."""
    n = len(m)
    a = [list(r) + [1 if i == j else 0 for j in range(n)] for i, r in enumerate(m)]
    for c in range(n):
        p = next((r for r in range(c, n) if a[r][c]), None)
        if p is None:
            raise ValueError("singular matrix")
        a[c], a[p] = a[p], a[c]
        inv = gf_inv(a[c][c])
        a[c] = [gf_mul(inv, v) for v in a[c]]
        for r in range(n):
            if r != c and a[r][c]:
                f = a[r][c]
                a[r] = [v ^ gf_mul(f, w) for v, w in zip(a[r], a[c])]
    return [r[n:] for r in a]


def vandermonde(rows, cols):
    return [[gf_exp(r, c) for c in range(cols)] for r in range(rows)]


_MATRIX_CACHE = {}


class CodingError(Exception):
    """ReedSolomon::new refused the shard counts (hbbft: Error::CodingNewReedSolomon)."""


def check_counts(k, p):
    """ReedSolomon::new: TooFewDataShards / TooFewParityShards / TooManyShards (> 256: the
    field has 256 elements, so hbbft's Broadcast::new fails for more than 256 nodes)."""
    if k == 0:
        raise CodingError("TooFewDataShards")
    if p == 0:
        raise CodingError("TooFewParityShards")
    if k + p > 256:
        raise CodingError("TooManyShards")


def build_matrix(k, n):
    """reed-solomon-erasure build_matrix(data_shards, total_shards)."""
    check_counts(k, n - k)
    key = (k, n)
    if key not in _MATRIX_CACHE:
        v = vandermonde(n, k)
        _MATRIX_CACHE[key] = mat_mul(v, mat_inv(v[:k]))
    return _MATRIX_CACHE[key]


def _apply(rows, inputs):
    """out[r] = sum_j rows[r][j] * inputs[j] (byte arrays)."""
    outs = []
    for row in rows:
        acc = np.zeros(len(inputs[0]), np.uint8)
        for c, x in zip(row, inputs):
            if c:
                acc ^= MUL[c, x]
        outs.append(acc)
    return outs


def rs_encode(shards, k, p):
    """ReedSolomon::encode: shards = k data + p parity byte strings of equal length; returns the
    k + p shards with the parity recomputed."""
    m = build_matrix(k, k + p)
    data = [np.frombuffer(bytes(s), np.uint8) for s in shards[:k]]
    parity = _apply(m[k:], data)
    return [bytes(s) for s in shards[:k]] + [bytes(x) for x in parity]


class ReconstructError(Exception):
    pass


def rs_reconstruct(shards, k, p):
    """ReedSolomon::reconstruct_shards: shards = list of bytes or None (length k + p); returns
    the completed list.  Raises ReconstructError (TooFewShardsPresent / IncorrectShardSize)."""
    n = k + p
    if len(shards) != n:
        raise ReconstructError("wrong shard count")
    present = [i for i, s in enumerate(shards) if s is not None]
    sizes = {len(shards[i]) for i in present}
    if len(sizes) > 1:
        raise ReconstructError("IncorrectShardSize")
    if len(present) == n:
        return list(shards)
    if len(present) < k:
        raise ReconstructError("TooFewShardsPresent")
    m = build_matrix(k, n)
    use = present[:k]
    dec = mat_inv([m[i] for i in use])
    sub = [np.frombuffer(bytes(shards[i]), np.uint8) for i in use]
    out = list(shards)
    missing_data = [i for i in range(k) if shards[i] is None]
    for i, v in zip(missing_data, _apply([dec[i] for i in missing_data], sub)):
        out[i] = bytes(v)
    data = [np.frombuffer(bytes(out[i]), np.uint8) for i in range(k)]
    missing_par = [i for i in range(k, n) if shards[i] is None]
    for i, v in zip(missing_par, _apply([m[i] for i in missing_par], data)):
        out[i] = bytes(v)
    return out


# ------------------------------------------------------------------ Merkle tree (merkle.rs)
def sha3(b):
    return hashlib.sha3_256(bytes(b)).digest()


def merkle_levels(values):
    """MerkleTree::from_vec: the levels below the root (leaf digests first) and the root."""
    levels = []
    cur = [sha3(v) for v in values]
    while len(cur) > 1:
        nxt = [sha3(cur[i] + cur[i + 1]) if i + 1 < len(cur) else cur[i] for i in range(0, len(cur), 2)]
        levels.append(cur)
        cur = nxt
    return levels, cur[0]


def merkle_proof(levels, root, values, index):
    """MerkleTree::proof -> (value, index, digests, root)."""
    if index >= len(values):
        return None
    digests, i = [], index
    for lvl in levels:
        if (i ^ 1) < len(lvl):
            digests.append(lvl[i ^ 1])
        i //= 2
    return (bytes(values[index]), index, digests, root)


def proof_validate(proof, n):
    """Proof::validate(n)."""
    value, index, digests, root = proof
    d = sha3(value)
    i, m, it = index, n, 0
    while m > 1:
        if (i ^ 1) < m:
            if it >= len(digests):
                return False
            s = digests[it]
            it += 1
            d = sha3(s + d) if i & 1 else sha3(d + s)
        i //= 2
        m = (m + 1) // 2
    if it != len(digests):
        return False
    return d == root


# ------------------------------------------------------------------ broadcast.rs
def shard_counts(n_nodes, n_faulty):
    p = 2 * n_faulty
    return n_nodes - p, p


def send_shards(value, n_nodes, n_faulty):
    """Broadcast::send_shards: (shards, levels, root, proofs)."""
    k, p = shard_counts(n_nodes, n_faulty)
    v = struct.pack(">I", len(value)) + bytes(value)
    shard_len = (len(v) + k - 1) // k
    v = v + bytes(shard_len * (k + p) - len(v))
    shards = [v[i * shard_len:(i + 1) * shard_len] for i in range(k + p)]
    if p:
        shards = rs_encode(shards, k, p)
    levels, root = merkle_levels(shards)
    proofs = [merkle_proof(levels, root, shards, i) for i in range(len(shards))]
    return shards, levels, root, proofs


def glue_shards(values, k):
    data = b"".join(bytes(v) for v in values[:k])
    if len(data) < 4:
        return None
    n = struct.unpack(">I", data[:4])[0]
    return data[4:4 + n]


def decode_from_shards(leaf_values, n_faulty, root):
    """decode_from_shards: leaf_values = list (length N) of bytes or None."""
    n = len(leaf_values)
    k, p = shard_counts(n, n_faulty)
    try:
        if p:
            full = rs_reconstruct(leaf_values, k, p)
        else:
            if any(v is None for v in leaf_values):
                return None
            full = list(leaf_values)
    except ReconstructError:
        return None
    _, r = merkle_levels(full)
    if r != root:
        return None
    return glue_shards(full, k)
