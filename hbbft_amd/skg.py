"""SyncKeyGen batch queue — the host-side mirror of the reference's dealerless key generation
(/root/reference/src/sync_key_gen.rs:272-509) driving the GPU verifier.

The reference handles every Part / Ack synchronously: decrypt our row (our value), bincode-decode
it, check it against the proposer's bivariate commitment — one BivarCommitment::row (Part) or
BivarCommitment::evaluate (Ack) per message, G1-MSM heavy.  Here messages queue in arrival order;
``flush`` then
  1. decrypts every queued ciphertext addressed to us in one batch (SecretKey::decrypt:
     Ciphertext::verify + sk u + the hash_bytes pad; hbtc_decrypt),
  2. checks every decoded row in one hbtc_skg_check_parts call and every decoded value in one
     hbtc_skg_check_acks call (the value check of an Ack uses the commitment of the FIRST Part
     received from its proposer, the only one the reference ever stores, :346-354),
  3. replays the queue in order with those verdicts, so every state change and fault is the
     reference's: parts are stored before their row is checked (:346-354), an Ack is recorded in
     ``acks`` before its value is checked (:474-476), and the fault order is NodeCount ->
     SenderExist -> DuplicateAck -> ValueDecryption -> ValueDeserialization -> ValueInvalid
     (:467-495); a Part whose row fails to decrypt yields no outcome (the `?` at :358), one whose
     row does not decode or match yields InvalidPartMessage (:359-370),
  4. encrypts the Ack values of every valid Part in one batch (:372-380).
Verdicts depend only on the message and the stored commitment, never on later state, so the
replay reproduces the sequential outcomes exactly (tests/test_gpu_skg_protocol.py checks this
against oracle/hbbft_rules.py's line-by-line restatement).

Keys: ``generate`` (:428-447) sums row(0) of the complete Parts' commitments (one batched G1 MSM)
and interpolates our secret share; ``public_key_shares`` is Commitment::evaluate(i + 1) for
every node (hbtc_commitment_evaluate; NetworkInfo::new, src/messaging.rs:253-256).
Values on the wire use hbbft_amd/wire.py's bincode framing (parity-unpinned Fr layout).
"""
import secrets
from collections import namedtuple

import numpy as np

from . import _native as N
from . import wire

R = wire.R
G1_GEN = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G1_INF = bytes([0xC0]) + bytes(47)

Ciphertext = namedtuple("Ciphertext", "u v w")   # threshold_crypto Ciphertext(U, V, W)
Part = namedtuple("Part", "commit rows")         # sync_key_gen.rs:201: (BivarCommitment, rows)
Ack = namedtuple("Ack", "proposer values")       # sync_key_gen.rs:218: (proposer index, values)


def coeff_pos(i, j):
    """Index of coefficient (i, j) of a symmetric bivariate polynomial (packed upper triangle)."""
    return j * (j + 1) // 2 + i if j >= i else i * (i + 1) // 2 + j


def _fr_le(vals):
    return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals), np.uint8).copy()


# ------------------------------------------------------------------------------ encryption
def encrypt_batch(ctx, pks, msgs, rs=None):
    """PublicKey::encrypt_with_rng for n (pk_i, msg_i): u = r G1, v = msg XOR hash_bytes(r pk),
    w = r hash_g1_g2(u, v).  The group work runs batched on the GPU, the pads on the host."""
    n = len(msgs)
    if n == 0:
        return []
    rs = rs or [secrets.randbelow(R - 1) + 1 for _ in range(n)]
    sc = _fr_le(rs)
    u, st1 = ctx.g1_mul(G1_GEN, sc)
    g, st2 = ctx.g1_mul([bytes(p) for p in pks], sc)
    if st1.any() or st2.any():
        raise N.HbtcError("encrypt: a public key failed to decode")
    us = [bytes(u[48 * i:48 * i + 48]) for i in range(n)]
    gs = [bytes(g[48 * i:48 * i + 48]) for i in range(n)]
    vs = N.xor_hash_bytes_batch(gs, msgs)
    H = ctx.hash_g1_g2_batch(us, vs)
    w, st3 = ctx.g2_mul(H, sc)
    if st3.any():
        raise N.HbtcError("encrypt: hash point failed to decode")
    return [Ciphertext(us[i], vs[i], bytes(w[96 * i:96 * i + 96])) for i in range(n)]


def decrypt_batch(ctx, sk, cts):
    """SecretKey::decrypt for n ciphertexts under one key (hbtc_decrypt): None where
    Ciphertext::verify fails (or u / w does not decode), else v XOR hash_bytes(sk u)."""
    if not cts:
        return []
    pts, _ = ctx.decrypt(sk, [bytes(c.u) for c in cts], [bytes(c.w) for c in cts],
                         [bytes(c.v) for c in cts])
    return pts


# ------------------------------------------------------------------------------ SyncKeyGen
class _Proposal:
    """ProposalState (:231-254): the commitment, the verified values, the acking nodes."""

    def __init__(self, commit):
        self.commit = commit
        self.values = {}       # sender_idx + 1 -> Fr
        self.acks = set()
        self.our_row = None    # our row, once it matched the commitment (fast Ack check)

    def is_complete(self, t):
        return len(self.acks) > 2 * t


class SyncKeyGen:
    """One node's SyncKeyGen instance with batched message handling (see module docstring)."""

    def __init__(self, ctx, our_id, sec_key, pub_keys, threshold):
        self.ctx = ctx
        self.our_id = our_id
        self.sec_key = int(sec_key)
        self.ids = sorted(pub_keys)
        self.pub_keys = {i: bytes(pub_keys[i]) for i in self.ids}
        self.index = {n: i for i, n in enumerate(self.ids)}
        self.our_idx = self.index.get(our_id)
        self.t = int(threshold)
        self.parts = {}
        self.queue = []

    @classmethod
    def new(cls, ctx, our_id, sec_key, pub_keys, threshold):
        """SyncKeyGen::new (:293-330): the instance and our Part (None for an observer)."""
        kg = cls(ctx, our_id, sec_key, pub_keys, threshold)
        if kg.our_idx is None:
            return kg, None
        t = kg.t
        b = [secrets.randbelow(R) for _ in range((t + 1) * (t + 2) // 2)]  # BivarPoly::random
        cm, st = ctx.g1_mul(G1_GEN, _fr_le(b))
        if st.any():
            raise N.HbtcError("commitment failed")
        commit = [bytes(cm[48 * i:48 * i + 48]) for i in range(len(b))]
        rows = [wire.poly_to_wire(_bivar_row(b, t, i + 1)) for i in range(len(kg.ids))]
        cts = encrypt_batch(ctx, [kg.pub_keys[n] for n in kg.ids], rows)
        return kg, Part(commit, cts)

    # ---------------------------------------------------------------- queue
    def handle_part(self, sender_id, part):
        self.queue.append(("part", sender_id, part))

    def handle_ack(self, sender_id, ack):
        self.queue.append(("ack", sender_id, ack))

    def flush(self):
        """Process the queue; one result per queued message, in order:
        Part -> None | ("valid", Ack) | ("invalid", [(sender, "InvalidPartMessage")]);
        Ack  -> list of faults [(sender, ("AckMessage", fault))] (empty when handled)."""
        q, self.queue = self.queue, []
        n, t, our = len(self.ids), self.t, self.our_idx
        # 1. ciphertexts addressed to us (stateless pre-pass)
        jobs = []
        for m, (kind, sender, msg) in enumerate(q):
            if our is None or sender not in self.index:
                continue
            cts = msg.rows if kind == "part" else msg.values
            if kind == "ack" and len(cts) != n:
                continue  # NodeCount: nothing to decrypt
            if our < len(cts):
                jobs.append((m, cts[our]))
        plain = dict(zip([m for m, _ in jobs], decrypt_batch(self.ctx, self.sec_key, [c for _, c in jobs])))
        # 2. decode; the commitment each message is checked against (first Part per proposer)
        rows, vals, commit_of = {}, {}, {}
        first_part = {p: st.commit for p, st in self.parts.items()}
        for m, (kind, sender, msg) in enumerate(q):
            if sender not in self.index:
                continue
            if kind == "part":
                s_idx = self.index[sender]
                if s_idx not in first_part:
                    first_part[s_idx] = msg.commit
                    commit_of[m] = msg.commit
                if m in plain and plain[m] is not None:
                    try:
                        row = wire.poly_from_wire(plain[m])
                        rows[m] = row if len(row) == t + 1 else None
                    except wire.WireError:
                        rows[m] = None
            else:
                if m in plain and plain[m] is not None:
                    try:
                        vals[m] = wire.fr_value_from_wire(plain[m])
                    except wire.WireError:
                        vals[m] = None
                if msg.proposer in first_part:
                    commit_of[m] = first_part[msg.proposer]
        # 3. batched checks: rows of the stored Parts, values of every decodable Ack
        row_ok = {}
        pm = [m for m in rows if rows[m] is not None and m in commit_of]
        if pm:
            st = self.ctx.skg_check_parts(t, our, [p for m in pm for p in commit_of[m]],
                                          [rows[m] for m in pm])
            row_ok = {m: int(st[i]) == N.ACCEPT for i, m in enumerate(pm)}
        val_ok = {}
        am = [m for m in vals if vals[m] is not None and m in commit_of]
        if am:
            val_ok = self._check_values(q, am, vals, commit_of, rows, row_ok)
        # 4. replay in order
        out, new_acks = [], []
        for m, (kind, sender, msg) in enumerate(q):
            if kind == "part":
                out.append(self._replay_part(m, sender, msg, plain, rows, row_ok, new_acks))
            else:
                out.append(self._replay_ack(m, sender, msg, plain, vals, val_ok))
        self._emit_acks(new_acks, out)
        return out

    def _check_values(self, q, am, vals, commit_of, rows, row_ok):
        t, our = self.t, self.our_idx
        keys, commits, prow, pok = {}, [], [], []
        for m in am:
            c = commit_of[m]
            key = id(c)
            if key not in keys:
                keys[key] = len(commits)
                commits.append(c)
                # our verified row for this commitment, if we have one: the scalar fast path
                row = None
                for st in self.parts.values():
                    if st.commit is c and st.our_row is not None:
                        row = st.our_row
                for mm, r in rows.items():
                    if row is None and r is not None and row_ok.get(mm) and commit_of.get(mm) is c:
                        row = r
                prow.append(row if row is not None else [0] * (t + 1))
                pok.append(1 if row is not None else 0)
        ack_part = [keys[id(commit_of[m])] for m in am]
        ack_sender = [self.index[q[m][1]] for m in am]
        st = self.ctx.skg_check_acks(t, our, [p for c in commits for p in c], prow, pok, ack_part,
                                     ack_sender, [vals[m] for m in am])
        return {m: int(st[i]) == N.ACCEPT for i, m in enumerate(am)}

    def _replay_part(self, m, sender, part, plain, rows, row_ok, new_acks):  # :338-381
        if sender not in self.index:
            return None
        s_idx = self.index[sender]
        if s_idx in self.parts:
            return None  # multiple parts: ignored
        st = _Proposal(part.commit)
        self.parts[s_idx] = st
        if self.our_idx is None:
            return None
        if self.our_idx >= len(part.rows) or plain.get(m) is None:
            return None  # rows.get(our_idx)? / decrypt(..)?
        if rows.get(m) is None or not row_ok.get(m, False):
            return ("invalid", [(sender, "InvalidPartMessage")])
        st.our_row = rows[m]
        new_acks.append((m, s_idx, rows[m]))
        return ("valid", None)  # the Ack is filled in by _emit_acks

    def _replay_ack(self, m, sender, ack, plain, vals, val_ok):  # :387-396, :462-498
        if sender not in self.index:
            return []
        s_idx = self.index[sender]

        def fault(kind):
            return [(sender, ("AckMessage", kind))]
        if len(ack.values) != len(self.ids):
            return fault("NodeCount")
        st = self.parts.get(ack.proposer)
        if st is None:
            return fault("SenderExist")
        if s_idx in st.acks:
            return fault("DuplicateAck")
        st.acks.add(s_idx)
        if self.our_idx is None:
            return []
        if plain.get(m) is None:
            return fault("ValueDecryption")
        if vals.get(m) is None:
            return fault("ValueDeserialization")
        if not val_ok.get(m, False):  # checked against this (the stored) commitment
            return fault("ValueInvalid")
        st.values[s_idx + 1] = vals[m]
        return []

    def _emit_acks(self, new_acks, out):
        """Ack(sender_idx, values): row(idx + 1) encrypted to every node (:371-380), batched."""
        if not new_acks:
            return
        n = len(self.ids)
        msgs, pks = [], []
        for _, _, row in new_acks:
            for i in range(n):
                msgs.append(wire.fr_to_wire(_poly_eval(row, i + 1)))
                pks.append(self.pub_keys[self.ids[i]])
        cts = encrypt_batch(self.ctx, pks, msgs)
        for a, (m, s_idx, _) in enumerate(new_acks):
            out[m] = ("valid", Ack(s_idx, cts[a * n:(a + 1) * n]))

    # ---------------------------------------------------------------- keys
    def count_complete(self):
        return sum(1 for st in self.parts.values() if st.is_complete(self.t))

    def is_node_ready(self, proposer_id):
        st = self.parts.get(self.index.get(proposer_id))
        return bool(st and st.is_complete(self.t))

    def is_ready(self):
        return self.count_complete() > self.t

    def generate(self):
        """(public key set commitment [t+1 compressed G1], our secret key share or None)."""
        t = self.t
        done = [self.parts[p] for p in sorted(self.parts) if self.parts[p].is_complete(t)]
        if done:
            pts = [st.commit[coeff_pos(0, j)] for j in range(t + 1) for st in done]
            commit, st = self.ctx.g1_msm(t + 1, len(done), pts, [1] * len(pts))
            if st.any():
                raise N.HbtcError("generate: a commitment point failed to decode")
        else:
            commit = []  # Poly::zero().commitment(): no coefficients
        sk = None
        if self.our_idx is not None:
            sk = 0
            for st in done:  # Poly::interpolate(values.take(t + 1)).evaluate(0)
                sk = (sk + _lagrange_at_zero(sorted(st.values.items())[:t + 1])) % R
        return commit, sk

    def public_key_shares(self, commit):
        """public_key_share(i) = commitment.evaluate(i + 1) for every node (messaging.rs:253-256)."""
        pks, st = self.ctx.commitment_evaluate(commit, [i + 1 for i in range(len(self.ids))])
        if st.any():
            raise N.HbtcError("public key shares: commitment failed to decode")
        return pks


def _poly_eval(coeffs, x):
    acc = 0
    for c in reversed(coeffs):
        acc = (acc * x + c) % R
    return acc


def _bivar_row(b, t, x):
    xp = [pow(x, j, R) for j in range(t + 1)]
    return [sum(b[coeff_pos(i, j)] * xp[j] for j in range(t + 1)) % R for i in range(t + 1)]


def _lagrange_at_zero(items):
    """Poly::interpolate(items).evaluate(0) over (x, y) pairs with distinct x."""
    xs = [x % R for x, _ in items]
    acc = 0
    for x, y in items:
        num, den = 1, 1
        for x0 in xs:
            if x0 != x % R:
                num = num * x0 % R
                den = den * (x0 - x) % R
        acc = (acc + y * num * pow(den, R - 2, R)) % R
    return acc
