#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/*.json from the Python oracle.

The reference (threshold_crypto 0.1.0-rng-fix / pairing 0.14.2) cannot be built
or imported here, so the expected outputs come from the oracle's restatement of threshold_crypto
(oracle/threshold_crypto.py, every verify = two FULL pairings compared, exactly the reference's
algorithm) on seeded synthetic key sets shaped like hbbft's: sk_i = poly(i + 1) for a random
degree-f polynomial (NetworkInfo::generate_map, /root/reference/src/messaging.rs:361-402),
coin nonces in hbbft's Nonce format (src/binary_agreement/mod.rs:155-166), ciphertexts from
encrypt_with_rng semantics.  Corrupted items follow SURVEY.md §8d's corruption mix.

Run: python tests/golden/make_golden.py      (about a minute; writes c1_coin.json, c1_dec.json,
codec.json, multi_coin.json)
"""
import json
import os
import random
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import bls12_381 as B  # noqa: E402
from oracle import threshold_crypto as T  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SEED = 0x6862626674  # "hbbft"


def hx(b):
    return bytes(b).hex()


def keyset(rng, n):
    f = (n - 1) // 3
    coeffs = [rng.randrange(1, B.R) for _ in range(f + 1)]
    sks = [T.poly_evaluate(coeffs, i + 1) for i in range(n)]
    pks = [B.g1_mul(B.G1_GEN, s) for s in sks]
    master_sk = coeffs[0]
    master_pk = B.g1_mul(B.G1_GEN, master_sk)
    return f, coeffs, sks, pks, master_sk, master_pk


def non_subgroup_g1(rng):
    while True:
        p = B.g1_point_from_x(rng.randrange(B.P), rng.random() < 0.5)
        if p is not None and not B.g1_in_subgroup(p):
            return p


def non_subgroup_g2(rng):
    while True:
        p = B.g2_point_from_x((rng.randrange(B.P), rng.randrange(B.P)), rng.random() < 0.5)
        if p is not None and not B.g2_in_subgroup(p):
            return p


def off_curve_x(rng, group):
    """An x (< p) for which no point exists: a DECODE_ERR encoding."""
    while True:
        if group == 1:
            x = rng.randrange(B.P)
            if B.g1_point_from_x(x, False) is None:
                b = bytearray(x.to_bytes(48, "big"))
                b[0] |= 0x80
                return bytes(b)
        else:
            x = (rng.randrange(B.P), rng.randrange(B.P))
            if B.g2_point_from_x(x, False) is None:
                b = bytearray(x[1].to_bytes(48, "big") + x[0].to_bytes(48, "big"))
                b[0] |= 0x80
                return bytes(b)


def bad_encodings(rng, group, valid):
    """Encodings pairing 0.14's into_affine rejects (name, bytes)."""
    size = 48 if group == 1 else 96
    out = []
    b = bytearray(valid)
    b[0] &= 0x7F
    out.append(("no_compression_flag", bytes(b)))
    b = bytearray(size)
    b[0] = 0xC0
    b[-1] = 1
    out.append(("infinity_with_payload", bytes(b)))
    b = bytearray(B.P.to_bytes(48, "big") + (b"\x00" * (size - 48)))
    b[0] |= 0x80
    out.append(("x_not_reduced", bytes(b)))
    out.append(("not_on_curve", off_curve_x(rng, group)))
    ns = non_subgroup_g1(rng) if group == 1 else non_subgroup_g2(rng)
    out.append(("not_in_subgroup", B.g1_compress(ns) if group == 1 else B.g2_compress(ns)))
    return out


def coin_fixture(rng, n):
    f, coeffs, sks, pks, msk, mpk = keyset(rng, n)
    t = f + 1
    invocation = B.g1_compress(mpk)
    nonce = T.coin_nonce(invocation, 0, 2, 0)
    H = T.hash_g2(nonce)
    sigs = [B.g2_mul(H, s) for s in sks]
    items = []  # (name, idx, sig_bytes, expected)
    for i in range(n):
        items.append(("valid_%d" % i, i, B.g2_compress(sigs[i])))
    other = T.hash_g2(T.coin_nonce(invocation, 0, 2, 1))
    delta = B.g2_mul(B.G2_GEN, rng.randrange(1, B.R))
    items += [
        ("wrong_key", 1, B.g2_compress(sigs[0])),
        ("plus_generator", 2, B.g2_compress(B.g2_add(sigs[2], B.G2_GEN))),
        ("identity", 3, B.g2_compress(None)),
        ("wrong_message", 4, B.g2_compress(B.g2_mul(other, sks[4]))),
        ("cancel_a", 5 % n, B.g2_compress(B.g2_add(sigs[5 % n], delta))),
        ("cancel_b", 6 % n, B.g2_compress(B.g2_add(sigs[6 % n], B.g2_neg(delta)))),
        ("negated", 7 % n, B.g2_compress(B.g2_neg(sigs[7 % n]))),
        ("unknown_sender", n, B.g2_compress(sigs[0])),
    ]
    for name, enc in bad_encodings(rng, 2, B.g2_compress(sigs[0])):
        items.append(("enc_" + name, 0, enc))
    expected = []
    for name, idx, enc in items:
        if idx >= n:
            expected.append("UNKNOWN_SENDER")
            continue
        try:
            sig = B.g2_decompress(enc)
        except B.DecodeError:
            expected.append("DECODE_ERR")
            continue
        expected.append("ACCEPT" if T.verify_g2(pks[idx], sig, H) else "REJECT")
    # combines (A3 + A4 + A2): first t valid shares by index; another subset gives the same bytes
    first = [(i, sigs[i]) for i in range(t)]
    comb = T.combine_signatures(t, first)
    alt = [(i, sigs[i]) for i in range(n - t, n)]
    comb_alt = T.combine_signatures(t, alt)
    assert comb == comb_alt
    master_ok = T.verify_g2(mpk, comb, H)
    assert master_ok
    combines = [
        {"name": "first_t", "idx": [i for i, _ in first], "sigs": [hx(B.g2_compress(s)) for _, s in first],
         "expected": "ACCEPT", "sig": hx(B.g2_compress(comb)), "parity": int(T.signature_parity(comb))},
        {"name": "last_t", "idx": [i for i, _ in alt], "sigs": [hx(B.g2_compress(s)) for _, s in alt],
         "expected": "ACCEPT", "sig": hx(B.g2_compress(comb)), "parity": int(T.signature_parity(comb))},
        {"name": "duplicate", "idx": [0, 0] + list(range(1, t - 1)) if t > 2 else [0, 0],
         "sigs": [hx(B.g2_compress(sigs[0]))] * 2 + [hx(B.g2_compress(sigs[i])) for i in range(1, t - 1)],
         "expected": "DUPLICATE_ENTRY"},
        {"name": "not_enough", "idx": list(range(t - 1)),
         "sigs": [hx(B.g2_compress(sigs[i])) for i in range(t - 1)], "expected": "NOT_ENOUGH_SHARES"},
    ]
    return {
        "config": "C1 coin N=%d f=%d t=%d" % (n, f, t),
        "n": n, "f": f, "t": t,
        "pk_shares": [hx(B.g1_compress(p)) for p in pks],
        "master_pk": hx(B.g1_compress(mpk)),
        "nonce": hx(nonce),
        "H": hx(B.g2_compress(H)),
        "items": [{"name": nm, "idx": ix, "sig": hx(enc), "expected": ex}
                  for (nm, ix, enc), ex in zip(items, expected)],
        "combines": combines,
        "master_verify": bool(master_ok),
    }


def dec_fixture(rng, n):
    f, coeffs, sks, pks, msk, mpk = keyset(rng, n)
    t = f + 1
    r = rng.randrange(1, B.R)
    msg = bytes(rng.randrange(256) for _ in range(32))
    u, v, w = T.encrypt_with_rng(mpk, r, msg)
    H = T.hash_g1_g2(u, v)
    assert T.ciphertext_verify_h(u, H, w)
    shares = [B.g1_mul(u, s) for s in sks]
    items = [("valid_%d" % i, i, B.g1_compress(shares[i])) for i in range(n)]
    delta = B.g1_mul(B.G1_GEN, rng.randrange(1, B.R))
    items += [
        ("wrong_key", 1, B.g1_compress(shares[0])),
        ("plus_generator", 2, B.g1_compress(B.g1_add(shares[2], B.G1_GEN))),
        ("identity", 3, B.g1_compress(None)),
        ("cancel_a", 5 % n, B.g1_compress(B.g1_add(shares[5 % n], delta))),
        ("cancel_b", 6 % n, B.g1_compress(B.g1_add(shares[6 % n], B.g1_neg(delta)))),
        ("negated", 7 % n, B.g1_compress(B.g1_neg(shares[7 % n]))),
        ("unknown_sender", n, B.g1_compress(shares[0])),
    ]
    for name, enc in bad_encodings(rng, 1, B.g1_compress(shares[0])):
        items.append(("enc_" + name, 0, enc))
    expected = []
    for name, idx, enc in items:
        if idx >= n:
            expected.append("UNKNOWN_SENDER")
            continue
        try:
            d = B.g1_decompress(enc)
        except B.DecodeError:
            expected.append("DECODE_ERR")
            continue
        expected.append("ACCEPT" if T.verify_decryption_share_h(pks[idx], d, H, w) else "REJECT")
    first = [(i, shares[i]) for i in range(t)]
    plain, g = T.decrypt(t, first, (u, v, w))
    assert plain == msg
    alt = [(i, shares[i]) for i in range(n - t, n)]
    _, g_alt = T.decrypt(t, alt, (u, v, w))
    assert g == g_alt
    bad_w = B.g2_add(w, B.G2_GEN)
    return {
        "config": "C1-size HoneyBadger ciphertext N=%d f=%d t=%d" % (n, f, t),
        "n": n, "f": f, "t": t,
        "pk_shares": [hx(B.g1_compress(p)) for p in pks],
        "master_pk": hx(B.g1_compress(mpk)),
        "u": hx(B.g1_compress(u)), "v": hx(v), "w": hx(B.g2_compress(w)),
        "H": hx(B.g2_compress(H)),
        "plaintext": hx(msg),
        "items": [{"name": nm, "idx": ix, "share": hx(enc), "expected": ex}
                  for (nm, ix, enc), ex in zip(items, expected)],
        "combines": [
            {"name": "first_t", "idx": [i for i, _ in first],
             "shares": [hx(B.g1_compress(s)) for _, s in first], "expected": "ACCEPT",
             "g": hx(B.g1_compress(g))},
            {"name": "last_t", "idx": [i for i, _ in alt],
             "shares": [hx(B.g1_compress(s)) for _, s in alt], "expected": "ACCEPT",
             "g": hx(B.g1_compress(g))},
        ],
        "ciphertext_checks": [
            {"name": "valid", "u": hx(B.g1_compress(u)), "H": hx(B.g2_compress(H)),
             "w": hx(B.g2_compress(w)), "expected": "ACCEPT"},
            {"name": "w_plus_generator", "u": hx(B.g1_compress(u)), "H": hx(B.g2_compress(H)),
             "w": hx(B.g2_compress(bad_w)), "expected": "REJECT"},
        ],
    }


def codec_fixture(rng):
    """Known-answer encodings: public generator encodings of the BLS12-381 / zcash spec, and
    k*G for a few k (decode, re-encode, scalar-mult reference values)."""
    ks = [1, 2, 3, B.R - 1, rng.randrange(B.R), rng.randrange(B.R)]
    return {
        "g1_generator": hx(B.g1_compress(B.G1_GEN)),
        "g2_generator": hx(B.g2_compress(B.G2_GEN)),
        "g1_mul": [{"k": "%064x" % k, "out": hx(B.g1_compress(B.g1_mul(B.G1_GEN, k)))} for k in ks],
        "g2_mul": [{"k": "%064x" % k, "out": hx(B.g2_compress(B.g2_mul(B.G2_GEN, k)))} for k in ks],
        "g1_bad": [{"name": nm, "enc": hx(e)} for nm, e in bad_encodings(rng, 1, B.g1_compress(B.G1_GEN))],
        "g2_bad": [{"name": nm, "enc": hx(e)} for nm, e in bad_encodings(rng, 2, B.g2_compress(B.G2_GEN))],
    }


def multi_coin_fixture(rng, n, n_inst):
    """Several coin instances in one batch, with uneven share counts (incl. an empty one)."""
    f, coeffs, sks, pks, msk, mpk = keyset(rng, n)
    invocation = B.g1_compress(mpk)
    insts = []
    for k in range(n_inst):
        nonce = T.coin_nonce(invocation, 3, 2, k)
        H = T.hash_g2(nonce)
        cnt = [n, 0, 3, n - 1][k % 4]
        senders = rng.sample(range(n), cnt)
        items = []
        for j, i in enumerate(senders):
            s = B.g2_mul(H, sks[i])
            bad = (j == 1)
            if bad:
                s = B.g2_add(s, B.G2_GEN)
            items.append({"idx": i, "sig": hx(B.g2_compress(s)), "expected": "REJECT" if bad else "ACCEPT"})
        insts.append({"nonce": hx(nonce), "H": hx(B.g2_compress(H)), "items": items})
    return {"n": n, "pk_shares": [hx(B.g1_compress(p)) for p in pks], "instances": insts}


def main():
    rng = random.Random(SEED)
    fixtures = {
        "codec.json": codec_fixture(rng),
        "c1_coin.json": coin_fixture(rng, 10),
        "c1_dec.json": dec_fixture(rng, 10),
        "multi_coin.json": multi_coin_fixture(rng, 7, 5),
    }
    for name, data in fixtures.items():
        with open(os.path.join(OUT, name), "w") as fh:
            json.dump(data, fh, indent=1)
        print("wrote", name)


if __name__ == "__main__":
    main()
