"""The oracle itself, on CPU: pinned to public known answers, cross-checked between its two
independent restatements (Python big-int: oracle/bls12_381.py + threshold_crypto.py; C 64-bit
limbs with pairing 0.14's algorithms: oracle/c/tc_oracle.c), and against the golden fixtures."""
import hashlib
import json
import os
import random

import pytest

from oracle import bls12_381 as B
from oracle import threshold_crypto as T

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# Public BLS12-381 / zcash-serialization known answers (not derived from this repo's code)
G1_GEN_COMPRESSED = ("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G2_GEN_COMPRESSED = ("93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
                     "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")


def fx(name):
    with open(os.path.join(GOLDEN, name)) as fh:
        return json.load(fh)


def test_known_answer_constants():
    assert B.R == 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    assert B.P.bit_length() == 381 and B.R.bit_length() == 255
    assert B.g1_compress(B.G1_GEN).hex() == G1_GEN_COMPRESSED
    assert B.g2_compress(B.G2_GEN).hex() == G2_GEN_COMPRESSED
    assert B.on_curve(B.FQ, B.G1_GEN) and B.on_curve(B.FQ2, B.G2_GEN)
    assert B.g1_mul(B.G1_GEN, B.R) is None and B.g2_mul(B.G2_GEN, B.R) is None


def test_python_pairing_bilinear_and_nondegenerate():
    rng = random.Random(11)
    a, b = rng.randrange(1, B.R), rng.randrange(1, B.R)
    e = B.pairing(B.G1_GEN, B.G2_GEN)
    assert e != B.f12_one()
    assert B.pairing(B.g1_mul(B.G1_GEN, a), B.g2_mul(B.G2_GEN, b)) == \
        B.pairing(B.g1_mul(B.G1_GEN, a * b % B.R), B.G2_GEN)


def test_golden_codec_matches_python_oracle():
    d = fx("codec.json")
    assert d["g1_generator"] == G1_GEN_COMPRESSED and d["g2_generator"] == G2_GEN_COMPRESSED
    for e in d["g1_mul"][:3]:
        assert B.g1_compress(B.g1_mul(B.G1_GEN, int(e["k"], 16))).hex() == e["out"]
    for e in d["g1_bad"] + d["g2_bad"]:
        dec = B.g1_decompress if len(e["enc"]) == 96 else B.g2_decompress
        with pytest.raises(B.DecodeError):
            dec(bytes.fromhex(e["enc"]))


def test_golden_combines_recompute_in_python():
    c = fx("c1_coin.json")
    comb = c["combines"][0]
    sig = T.combine_signatures(c["t"], [(i, B.g2_decompress(bytes.fromhex(s)))
                                        for i, s in zip(comb["idx"], comb["sigs"])])
    assert B.g2_compress(sig).hex() == comb["sig"]
    assert int(T.signature_parity(sig)) == comb["parity"]
    with pytest.raises(T.CryptoError):
        T.combine_signatures(c["t"], [(0, sig), (0, sig), (1, sig), (2, sig)])


# ---------------------------------------------------------------------- C restatement
cb = pytest.importorskip("oracle.cbaseline", reason="oracle/c not built (make oracle)")


def test_c_sha3_matches_hashlib():
    for n in (0, 1, 64, 135, 136, 137, 300):
        m = bytes(range(256))[:n] * 1 if n <= 256 else bytes(n)
        assert cb.sha3_256(m) == hashlib.sha3_256(m).digest()


def test_c_scalar_mul_and_codec_match_golden():
    d = fx("codec.json")
    g1, g2 = bytes.fromhex(d["g1_generator"]), bytes.fromhex(d["g2_generator"])
    for e in d["g1_mul"]:
        assert cb.g1_mul(g1, int(e["k"], 16)).hex() == e["out"]
    for e in d["g2_mul"]:
        assert cb.g2_mul(g2, int(e["k"], 16)).hex() == e["out"]
    for e in d["g1_bad"]:
        assert cb.g1_mul(bytes.fromhex(e["enc"]), 1) is None
    for e in d["g2_bad"]:
        assert cb.g2_mul(bytes.fromhex(e["enc"]), 1) is None


def test_c_hash_g2_matches_python_restatement():
    c = fx("c1_coin.json")
    nonce = bytes.fromhex(c["nonce"])
    assert cb.hash_g2(nonce).hex() == c["H"]
    for m in (b"", b"Help I'm trapped in a unit test factory"):
        assert cb.hash_g2(m) == B.g2_compress(T.hash_g2(m))
    d = fx("c1_dec.json")
    assert cb.hash_g1_g2(bytes.fromhex(d["u"]), bytes.fromhex(d["v"])).hex() == d["H"]
    long_msg = bytes(range(100))
    u = B.g1_decompress(bytes.fromhex(d["u"]))
    assert cb.hash_g1_g2(bytes.fromhex(d["u"]), long_msg) == B.g2_compress(T.hash_g1_g2(u, long_msg))


def test_c_pairing_decisions_match_golden():
    d = fx("c1_dec.json")
    H, w = bytes.fromhex(d["H"]), bytes.fromhex(d["w"])
    pks = [bytes.fromhex(p) for p in d["pk_shares"]]
    for it in d["items"]:
        if it["expected"] == "UNKNOWN_SENDER":
            continue
        r = cb.pairing_eq(bytes.fromhex(it["share"]), H, pks[it["idx"]], w)
        want = {"ACCEPT": True, "REJECT": False, "DECODE_ERR": None}[it["expected"]]
        assert r == want, it["name"]
    c = fx("c1_coin.json")
    Hc = bytes.fromhex(c["H"])
    g1 = bytes.fromhex(fx("codec.json")["g1_generator"])
    pks = [bytes.fromhex(p) for p in c["pk_shares"]]
    for it in c["items"][:14]:
        if it["expected"] == "UNKNOWN_SENDER":
            continue
        r = cb.pairing_eq(pks[it["idx"]], Hc, g1, bytes.fromhex(it["sig"]))
        assert r == {"ACCEPT": True, "REJECT": False, "DECODE_ERR": None}[it["expected"]], it["name"]


def test_c_combines_match_golden():
    c = fx("c1_coin.json")
    for comb in c["combines"]:
        st, out = cb.combine(2, comb["idx"], [bytes.fromhex(s) for s in comb["sigs"]], c["t"])
        want = {"ACCEPT": 0, "DUPLICATE_ENTRY": 6, "NOT_ENOUGH_SHARES": 5}[comb["expected"]]
        assert st == want
        if st == 0:
            assert out.hex() == comb["sig"]
            assert cb.sig_parity(out) == comb["parity"]
    d = fx("c1_dec.json")
    for comb in d["combines"]:
        st, out = cb.combine(1, comb["idx"], [bytes.fromhex(s) for s in comb["shares"]], d["t"])
        assert st == 0 and out.hex() == comb["g"]
