"""threshold_crypto @ 0.1.0-rng-fix restated in Python — TEST ORACLE ONLY.

The crate is a git dependency of hbbft (/root/reference/Cargo.toml:33, re-exported as
``crypto`` at src/lib.rs:136) and is NOT vendored, so every function below is a
restatement of its published semantics [EXT-UNVERIFIED], anchored on hbbft's call
sites:

  A1 ``PublicKeyShare::verify``              src/coin.rs:151, tests/sync_key_gen.rs:83
  A2 ``PublicKey::verify``                   src/coin.rs:192-197
  A3 ``PublicKeySet::combine_signatures``    src/coin.rs:185-191
  A4 ``Signature::parity``                   src/coin.rs:173
  A5 ``PublicKeyShare::verify_decryption_share``  src/threshold_decryption.rs:159
  A6 ``PublicKeySet::decrypt``               src/threshold_decryption.rs:181-185
  A7 ``SecretKeyShare::decrypt_share`` / ``Ciphertext::verify``  src/threshold_decryption.rs:98
  A8 ``SecretKeyShare::sign``                src/coin.rs:142
  A9 ``hash_g2`` / ``hash_g1_g2`` / ``hash_bytes`` (crate-internal)
  A10-A13 ``poly::{Poly, Commitment, BivarCommitment}``  src/sync_key_gen.rs:345,366,493; src/messaging.rs:255

Decisions (accept/reject, errors) and combined group elements are mathematically
determined and therefore pinned by the algebra; the hash byte streams depend on
``oracle.rand04`` and are parity-unpinned (see that module).
"""
import hashlib

from . import bls12_381 as B
from .rand04 import ChaChaRng

R_MONT = pow(2, 384, B.P)
R_MONT_INV = pow(R_MONT, B.P - 2, B.P)


def sha3_256(data):
    return hashlib.sha3_256(bytes(data)).digest()


def _seed_words(digest):
    return [int.from_bytes(digest[4 * i:4 * i + 4], "big") for i in range(8)]


# ----------------------------------------------------------------------------- A9 hashes
def fq_rand(rng):
    """ff_derive ``Rand for Fq``: 6 u64 limbs (limb 0 least significant), top 3 bits
    masked, rejection if >= p, and the limbs are a *Montgomery* representation."""
    while True:
        limbs = [rng.next_u64() for _ in range(6)]
        limbs[5] &= 0xFFFFFFFFFFFFFFFF >> 3
        rep = sum(l << (64 * i) for i, l in enumerate(limbs))
        if rep < B.P:
            return rep * R_MONT_INV % B.P


def fq2_rand(rng):
    c0 = fq_rand(rng)
    c1 = fq_rand(rng)
    return (c0, c1)


def g2_rand(rng):
    """pairing 0.14 ``Rand for G2``: x, greatest, get_point_from_x, scale_by_cofactor."""
    while True:
        x = fq2_rand(rng)
        greatest = rng.gen_bool()
        pt = B.g2_point_from_x(x, greatest)
        if pt is not None:
            q = B.g2_mul(pt, B.H2)
            if q is not None:
                return q


def hash_g2(msg):
    """``hash_g2``: sha3_256(msg) -> 8 big-endian u32 seed words -> ChaChaRng -> G2::rand."""
    return g2_rand(ChaChaRng(_seed_words(sha3_256(msg))))


def hash_g1_g2(g1, msg):
    """``hash_g1_g2``: msg (sha3'd if longer than 64 bytes) || compressed(g1), then hash_g2."""
    msg = bytes(msg)
    m = sha3_256(msg) if len(msg) > 64 else msg
    return hash_g2(m + B.g1_compress(g1))


def hash_bytes(g1, length):
    """``hash_bytes``: ChaChaRng seeded by sha3_256(compressed(g1)); ``length`` u8 draws."""
    rng = ChaChaRng(_seed_words(sha3_256(B.g1_compress(g1))))
    return bytes(rng.gen_u8() for _ in range(length))


# ----------------------------------------------------------------------------- verify
def verify_g2(pk, sig, h):
    """``PublicKey::verify_g2``: e(pk, H) == e(G1, sig) — two full pairings compared."""
    return B.pairing(pk, h) == B.pairing(B.G1_GEN, sig)


def verify(pk, sig, msg):
    """A1/A2 ``PublicKeyShare::verify`` / ``PublicKey::verify``."""
    return verify_g2(pk, sig, hash_g2(msg))


def verify_decryption_share_h(pk, share, h, w):
    """A5 with H = hash_g1_g2(u, v) precomputed: e(share, H) == e(pk, w)."""
    return B.pairing(share, h) == B.pairing(pk, w)


def verify_decryption_share(pk, share, ct):
    u, v, w = ct
    return verify_decryption_share_h(pk, share, hash_g1_g2(u, v), w)


def ciphertext_verify_h(u, h, w):
    """A7 ``Ciphertext::verify``: e(G1, w) == e(u, H)."""
    return B.pairing(B.G1_GEN, w) == B.pairing(u, h)


def ciphertext_verify(ct):
    u, v, w = ct
    return ciphertext_verify_h(u, hash_g1_g2(u, v), w)


# ----------------------------------------------------------------------------- producers
def sign(sk, msg):
    """A8 ``SecretKeyShare::sign``: sk * hash_g2(msg)."""
    return B.g2_mul(hash_g2(msg), sk)


def encrypt_with_rng(pk, r, msg):
    """``PublicKey::encrypt_with_rng`` with the scalar r supplied by the caller."""
    u = B.g1_mul(B.G1_GEN, r)
    g = B.g1_mul(pk, r)
    msg = bytes(msg)
    v = bytes(a ^ b for a, b in zip(hash_bytes(g, len(msg)), msg))
    w = B.g2_mul(hash_g1_g2(u, v), r)
    return (u, v, w)


def decrypt_share(sk, ct):
    """A7 ``SecretKeyShare::decrypt_share``: None unless ct verifies, else sk * u."""
    if not ciphertext_verify(ct):
        return None
    return B.g1_mul(ct[0], sk)


# ----------------------------------------------------------------------------- A3/A6 combine
class CryptoError(Exception):
    pass


def interpolate(t, items, group):
    """``interpolate(t, items)``: first t items in iteration order, x = idx + 1 in Fr;
    NotEnoughShares if fewer than t; DuplicateEntry when an x repeats (checked in
    order while accumulating); result = sum lambda_i * sample_i."""
    samples = [((idx + 1) % B.R, pt) for idx, pt in list(items)[:t]]
    if len(samples) < t:
        raise CryptoError("NotEnoughShares")
    mul, add = (B.g1_mul, B.g1_add) if group == 1 else (B.g2_mul, B.g2_add)
    result = None
    seen = []
    for x, sample in samples:
        if x in seen:
            raise CryptoError("DuplicateEntry")
        seen.append(x)
        l0 = 1
        for x0, _ in samples:
            if x0 != x:
                l0 = l0 * x0 % B.R * pow((x0 - x) % B.R, B.R - 2, B.R) % B.R
        result = add(result, mul(sample, l0))
    return result


def lagrange_at_zero(xs):
    """lambda_i(0) for distinct Fr abscissae xs (helper for fixtures)."""
    out = []
    for x in xs:
        l0 = 1
        for x0 in xs:
            if x0 != x:
                l0 = l0 * x0 % B.R * pow((x0 - x) % B.R, B.R - 2, B.R) % B.R
        out.append(l0)
    return out


def combine_signatures(t, items):
    """A3 ``PublicKeySet::combine_signatures`` (t = threshold + 1)."""
    return interpolate(t, items, 2)


def decrypt(t, items, ct):
    """A6 ``PublicKeySet::decrypt``: interpolate in G1, then v XOR hash_bytes(g, |v|)."""
    g = interpolate(t, items, 1)
    v = ct[1]
    return bytes(a ^ b for a, b in zip(hash_bytes(g, len(v)), v)), g


def signature_parity(sig):
    """A4 ``Signature::parity``: popcount parity of the XOR of the 192 uncompressed bytes."""
    x = 0
    for b in B.g2_uncompress_bytes(sig):
        x ^= b
    return bin(x).count("1") % 2 == 1


# ----------------------------------------------------------------------------- polynomials
def poly_evaluate(coeffs, x):
    """``Poly::evaluate`` (Horner over Fr)."""
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % B.R
    return acc


def commitment(coeffs):
    """``Poly::commitment``: coeff_k * G1."""
    return [B.g1_mul(B.G1_GEN, c) for c in coeffs]


def commitment_evaluate(commit, x):
    """``Commitment::evaluate`` (A13; messaging.rs:255 via public_key_share(idx) at x=idx+1)."""
    acc = None
    for c in reversed(commit):
        acc = B.g1_add(B.g1_mul(acc, x), c) if acc is not None else c
    return acc


def coeff_pos(i, j):
    """Position of coefficient (i, j) of a symmetric bivariate polynomial (i <= j)."""
    if j >= i:
        return j * (j + 1) // 2 + i
    return i * (i + 1) // 2 + j


def bivar_commitment_row(bcommit, degree, x):
    """A10 ``BivarCommitment::row(x)``: row_i = sum_j C_{ij} x^j, i = 0..degree."""
    xp = [pow(x, j, B.R) for j in range(degree + 1)]
    return [B.g1_sum([B.g1_mul(bcommit[coeff_pos(i, j)], xp[j]) for j in range(degree + 1)])
            for i in range(degree + 1)]


def bivar_commitment_evaluate(bcommit, degree, x, y):
    """A12 ``BivarCommitment::evaluate(x, y)`` = sum_{i,j} C_{ij} x^i y^j."""
    xp = [pow(x, j, B.R) for j in range(degree + 1)]
    yp = [pow(y, j, B.R) for j in range(degree + 1)]
    return B.g1_sum([B.g1_mul(bcommit[coeff_pos(i, j)], xp[i] * yp[j] % B.R)
                     for i in range(degree + 1) for j in range(degree + 1)])


def bivar_poly_row(bcoeffs, degree, x):
    """``BivarPoly::row(x)`` over Fr."""
    xp = [pow(x, j, B.R) for j in range(degree + 1)]
    return [sum(bcoeffs[coeff_pos(i, j)] * xp[j] for j in range(degree + 1)) % B.R
            for i in range(degree + 1)]


# ----------------------------------------------------------------------------- hbbft nonce
def coin_nonce(invocation_id, session_id, ba_epoch, proposer_id):
    """``Nonce::new`` (src/binary_agreement/mod.rs:155-166):
    format!("Nonce for Honey Badger {:?}@{}:{}:{}", invocation_id, session_id, ba_epoch, proposer_id)
    where ``{:?}`` of a Vec<u8> prints ``[1, 2, 3]``."""
    dbg = "[" + ", ".join(str(b) for b in invocation_id) + "]"
    return ("Nonce for Honey Badger %s@%d:%d:%d" % (dbg, session_id, ba_epoch, proposer_id)).encode()
