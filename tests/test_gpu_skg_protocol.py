"""SyncKeyGen through the batch queue (hbbft_amd/skg.py) on the GPU.

1. The reference's own scenario, tests/sync_key_gen.rs:14-101, for the same node counts
   (1, 2, 3, 4, 8, 15): every node makes a Part; the first t + 1 Parts are handled by every
   node (all Valid); the Acks of nodes 0 .. 2t are handled by every node; every node is then
   ready, derives the same public key set, signs a message with its new secret key share; every
   SignatureShare verifies under its public key share (hbtc_verify_sig_shares, key shares from
   hbtc_commitment_evaluate), the combined signature (hbtc_combine_sigs over t + 1 shares)
   verifies under the master key (hbtc_verify_sigs).
2. Fault order: a crafted message sequence exercising every Part / Ack outcome of
   src/sync_key_gen.rs:338-498 (InvalidPartMessage, duplicate and unknown-sender Parts, an
   undecryptable row, NodeCount, SenderExist, DuplicateAck recorded before the value check,
   ValueDecryption, ValueDeserialization, ValueInvalid) gives exactly the outcomes of
   oracle/hbbft_rules.py's sequential restatement (checker crypto: the C / Python oracle),
   flushed at once and in two parts, and the same secret share and key-set commitment.
"""
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from hbbft_amd import skg, wire
from oracle import bls12_381 as B
from oracle import hbbft_rules as HR
from oracle import threshold_crypto as TC

pytestmark = pytest.mark.gpu
R = B.R
G1 = B.g1_compress(B.G1_GEN)


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    yield c
    c.close()


def _keys(ctx, rng, n):
    sks = [rng.randrange(1, R) for _ in range(n)]
    pk, st = ctx.g1_mul(G1, sks)
    assert not st.any()
    return sks, {i: bytes(pk[48 * i:48 * i + 48]) for i in range(n)}


@pytest.mark.timeout(300)
@pytest.mark.parametrize("node_num", [1, 2, 3, 4, 8, 15])
def test_reference_sync_key_gen_scenario(ctx, node_num):
    rng = random.Random(node_num)
    t = (node_num - 1) // 3
    sec_keys, pub_keys = _keys(ctx, rng, node_num)
    nodes, proposals = [], []
    for i in range(node_num):
        kg, part = skg.SyncKeyGen.new(ctx, i, sec_keys[i], pub_keys, t)
        nodes.append(kg)
        proposals.append(part)
    acks = []
    for sender_id, proposal in enumerate(proposals[:t + 1]):
        for node in nodes:
            node.handle_part(sender_id, proposal)
    for node_id, node in enumerate(nodes):
        outs = node.flush()
        assert all(o is not None and o[0] == "valid" for o in outs), outs
        if node_id <= 2 * t:
            acks += [(node_id, o[1]) for o in outs]
    for node in nodes:
        assert not node.is_ready()
        for sender_id, ack in acks:
            node.handle_ack(sender_id, ack)
        assert all(f == [] for f in node.flush())
        assert node.is_ready()
    pk_set, _ = nodes[0].generate()
    msg = b"Help I'm trapped in a unit test factory"
    H = N.hash_g2(msg)
    shares, sks = [], []
    for node in nodes:
        pks, sk = node.generate()
        assert pks == pk_set and sk is not None
        sks.append(sk)
    sig, st = ctx.g2_mul(H, sks)  # SecretKeyShare::sign = sk * hash_g2(msg)
    assert not st.any()
    pk_shares = nodes[0].public_key_shares(pk_set)
    ks, bad = ctx.keyset_load(pk_shares)
    assert bad == 0
    ctx.set_verify_mode(N.MODE_RLC)
    vst = ctx.verify_sig_shares(ks, [H], [node_num], np.arange(node_num, dtype=np.uint32), sig)
    assert (vst == N.ACCEPT).all()
    out, _, cst = ctx.combine_sigs([t + 1], np.arange(t + 1, dtype=np.uint32), sig[:96 * (t + 1)], t + 1)
    assert (cst == N.ACCEPT).all()
    assert (ctx.verify_sigs([pk_set[0]], [H], [out[0]]) == N.ACCEPT).all()
    # the public key shares are the key shares' public keys (messaging.rs:253-256)
    own, _ = ctx.g1_mul(G1, sks)
    assert b"".join(pk_shares) == bytes(own)
    ctx.keyset_free(ks)


# --------------------------------------------------------------------------- fault order
def _oracle_crypto(sk, t, our_idx):
    from oracle import cbaseline as C

    def decrypt(ct):
        H = C.hash_g1_g2(ct.u, ct.v)
        ok = C.pairing_eq(G1, ct.w, ct.u, H)
        if not ok:
            return None
        g = C.g1_mul(ct.u, sk)
        return bytes(a ^ b for a, b in zip(TC.hash_bytes(B.g1_decompress(g), len(ct.v)), ct.v))

    def row_matches(commit, row):
        pts = [B.g1_decompress(c) for c in commit]
        want = TC.bivar_commitment_row(pts, t, our_idx + 1)
        return [B.g1_compress(p) for p in want] == [B.g1_compress(p) for p in TC.commitment(row)]

    def value_matches(commit, sender_idx, val):
        pts = [B.g1_decompress(c) for c in commit]
        lhs = TC.bivar_commitment_evaluate(pts, t, our_idx + 1, sender_idx + 1)
        return B.g1_compress(lhs) == B.g1_compress(B.g1_mul(B.G1_GEN, val))

    return decrypt, row_matches, value_matches


def _bivar_eval(b, t, x, y):
    return sum(b[skg.coeff_pos(i, j)] * pow(x, i, R) * pow(y, j, R)
               for i in range(t + 1) for j in range(t + 1)) % R


def _messages(ctx, rng, n, t, our, pub_keys):
    """The crafted sequence: (kind, sender, message) with known polynomials."""
    pks = [pub_keys[i] for i in range(n)]
    polys = {p: [rng.randrange(R) for _ in range((t + 1) * (t + 2) // 2)] for p in range(4)}
    commits = {}
    for p, b in polys.items():
        cm, _ = ctx.g1_mul(G1, b)
        commits[p] = [bytes(cm[48 * i:48 * i + 48]) for i in range(len(b))]

    def part(p, tamper_row=False, bad_ct=False, short=False, extra=b""):
        rows = [skg._bivar_row(polys[p], t, i + 1) for i in range(n)]
        if tamper_row:
            rows[our][0] = (rows[our][0] + 1) % R
        ser = [wire.poly_to_wire(r) for r in rows]
        ser[our] += extra  # bytes after the last coefficient: ignored by bincode 1.0
        cts = skg.encrypt_batch(ctx, pks, ser)
        if bad_ct:
            c = cts[our]
            cts[our] = skg.Ciphertext(c.u, c.v, cts[(our + 1) % n].w)
        if short:
            cts = cts[:our]
        return skg.Part(commits[p], cts)

    def ack(sender, p, value=None, raw=None, bad_ct=False, count=None):
        vals = [wire.fr_to_wire(_bivar_eval(polys[p], t, sender + 1, i + 1)) for i in range(n)]
        if value is not None:
            vals[our] = wire.fr_to_wire(value)
        if raw is not None:
            vals[our] = raw
        cts = skg.encrypt_batch(ctx, pks, vals)
        if bad_ct:
            c = cts[our]
            cts[our] = skg.Ciphertext(c.u, bytes(c.v[:-1]) + bytes([c.v[-1] ^ 1]), c.w)
        if count is not None:
            cts = cts[:count]
        return skg.Ack(p, cts)

    good_val = _bivar_eval(polys[0], t, 1 + 1, our + 1)
    return [
        ("part", 0, part(0)),
        ("part", 1, part(1, tamper_row=True)),           # InvalidPartMessage
        ("part", 0, part(2)),                            # second Part from 0: ignored
        ("part", 9, part(0)),                            # unknown sender
        ("part", 3, part(3, bad_ct=True)),               # our row undecryptable: no outcome
        ("ack", 0, ack(0, 0)),                           # ok
        ("ack", 0, ack(0, 0)),                           # DuplicateAck
        ("ack", 1, ack(1, 0, count=n - 1)),              # NodeCount
        ("ack", 1, ack(1, 2)),                           # SenderExist (no Part from 2 yet)
        ("ack", 1, ack(1, 0, value=(good_val + 5) % R)),  # ValueInvalid (recorded in acks)
        ("ack", 1, ack(1, 0)),                           # DuplicateAck, though valid
        ("ack", 3, ack(3, 0, bad_ct=True)),              # ValueDecryption
        ("ack", 2, ack(2, 3, raw=b"\x21" + bytes(39))),  # ValueDeserialization (bad length)
        ("ack", 3, ack(3, 3, raw=wire.fr_to_wire(0)[:8] + (R + 1).to_bytes(32, "big"))),  # >= r
        ("ack", 2, ack(2, 0, raw=wire.fr_to_wire(_bivar_eval(polys[0], t, 3, our + 1))
                        + b"\x07\x07")),                 # ok: appended bytes ignored (bincode 1.0)
        ("part", 2, part(2, extra=b"\x01\x02\x03")),        # ok now, appended bytes ignored
        ("ack", 3, ack(3, 2)),                           # ok
        ("ack", 0, ack(0, 2)),                           # ok
        ("ack", 1, ack(1, 2)),                           # ok: Part 2 complete (3 > 2t acks)
        ("ack", 9, ack(1, 2)),                           # unknown sender: nothing
        ("part", 3, part(3, short=True)),                # second Part from 3: ignored
    ]


def _norm(kind, o):
    if kind == "part":
        return None if o is None else (o[0],) + (() if o[0] == "valid" else (o[1],))
    return o


@pytest.mark.timeout(300)
@pytest.mark.parametrize("split", [None, 7])
def test_fault_order_matches_sequential_rules(ctx, split):
    pytest.importorskip("oracle.cbaseline")
    rng = random.Random(31)
    n, t, our = 4, 1, 2
    sec_keys, pub_keys = _keys(ctx, rng, n)
    msgs = _messages(ctx, rng, n, t, our, pub_keys)
    ref = HR.SyncKeyGen(range(n), our, t, *_oracle_crypto(sec_keys[our], t, our))
    want = []
    for kind, sender, m in msgs:
        if kind == "part":
            want.append(_norm(kind, ref.handle_part(sender, (m.commit, m.rows))))
        else:
            want.append(ref.handle_ack(sender, (m.proposer, m.values)))
    node = skg.SyncKeyGen(ctx, our, sec_keys[our], pub_keys, t)
    got = []
    cuts = [0, split, len(msgs)] if split else [0, len(msgs)]
    for a, b in zip(cuts, cuts[1:]):
        for kind, sender, m in msgs[a:b]:
            (node.handle_part if kind == "part" else node.handle_ack)(sender, m)
        got += [_norm(msgs[a + i][0], o) for i, o in enumerate(node.flush())]
    assert got == want
    kinds = {f[0][1][1] for f in want if isinstance(f, list) and f}
    assert kinds == {"NodeCount", "SenderExist", "DuplicateAck", "ValueDecryption",
                     "ValueDeserialization", "ValueInvalid"}
    assert ("invalid", [(1, "InvalidPartMessage")]) in want
    # keys: same complete parts, same secret share; the key-set commitment is row(0) summed
    assert node.is_ready() == ref.is_ready()
    commit, sk = node.generate()
    assert sk == ref.secret_share()
    done = ref.complete()
    assert done == sorted(p for p, st in node.parts.items() if st.is_complete(t)) and done
    want_commit = []
    for j in range(t + 1):
        acc = None
        for p in done:
            pt = B.g1_decompress(ref.parts[p]["commit"][skg.coeff_pos(0, j)])
            acc = pt if acc is None else B.g1_add(acc, pt)
        want_commit.append(B.g1_compress(acc))
    assert commit == want_commit


def test_commitment_evaluate_matches_oracle(ctx):
    rng = random.Random(5)
    coeffs = [rng.randrange(R) for _ in range(7)]
    cm, _ = ctx.g1_mul(G1, coeffs)
    commit = [bytes(cm[48 * i:48 * i + 48]) for i in range(7)]
    xs = [1, 2, 3, 1000, 2 ** 32 - 1]
    got, st = ctx.commitment_evaluate(commit, xs)
    assert not st.any()
    for x, g in zip(xs, got):
        assert g == B.g1_compress(TC.commitment_evaluate([B.g1_decompress(c) for c in commit], x))


def test_decrypt_batch_matches_oracle(ctx):
    """hbtc_decrypt (SecretKey::decrypt over a batch): plaintexts of valid ciphertexts (short and
    > 64-byte messages: hash_g1_g2 hashes long v first), None for a ciphertext whose w does not
    match (Ciphertext::verify fails) and for an undecodable u."""
    rng = random.Random(44)
    sk = rng.randrange(1, R)
    pk, _ = ctx.g1_mul(G1, [sk])
    msgs = [bytes(rng.randrange(256) for _ in range(L)) for L in (0, 1, 40, 64, 65, 300)]
    cts = skg.encrypt_batch(ctx, [bytes(pk)] * len(msgs), msgs)
    # oracle: the same ciphertexts decrypt to the same messages with the Python restatement
    for m, c in zip(msgs[:3], cts[:3]):
        u = B.g1_decompress(c.u)
        g = B.g1_mul(u, sk)
        assert bytes(a ^ b for a, b in zip(TC.hash_bytes(g, len(c.v)), c.v)) == m
        assert TC.ciphertext_verify((u, c.v, B.g2_decompress(c.w)))
    bad_w = skg.Ciphertext(cts[2].u, cts[2].v, cts[3].w)
    bad_u = skg.Ciphertext(bytes([cts[1].u[0] & 0x7F]) + cts[1].u[1:], cts[1].v, cts[1].w)
    out, st = ctx.decrypt(sk, [c.u for c in cts + [bad_w, bad_u]], [c.w for c in cts + [bad_w, bad_u]],
                          [c.v for c in cts + [bad_w, bad_u]])
    assert out[:len(msgs)] == msgs
    assert out[-2] is None and st[-2] == N.REJECT
    assert out[-1] is None and st[-1] == N.DECODE_ERR
