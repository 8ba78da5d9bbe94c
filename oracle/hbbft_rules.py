"""hbbft's Coin and ThresholdDecryption decision rules restated sequentially — TEST ORACLE ONLY.

A line-by-line restatement of the reference's per-message logic, verifying
each share the moment the reference would, through an injected verifier (the Python or C
oracle).  tests/ compare the product's batched replay (hbbft_amd/protocol.py) against it.

  Coin                 /root/reference/src/coin.rs:89-207
  ThresholdDecryption  /root/reference/src/threshold_decryption.rs:64-188

Events are tuples: ("input",) | ("msg", sender_id, share) for Coin, and ("ct", ct) |
("msg", sender_id, share) for ThresholdDecryption.  Each handler returns a Step dict
{"faults": [(id, kind)], "output": value-or-None, "error": name-or-None}.
"""


def _step(faults=None, output=None, error=None):
    return {"faults": list(faults or []), "output": output, "error": error}


class Coin:
    """coin.rs:64 — verify(sender, share) -> bool and combine(shares_by_index) -> (sig, parity)
    or raises; master_ok(sig) -> bool are injected."""

    def __init__(self, node_ids, our_id, num_faulty, our_share, verify, combine_and_parity,
                 master_verify):
        self.ids = sorted(node_ids)
        self.index = {n: i for i, n in enumerate(self.ids)}
        self.our_id = our_id
        self.f = num_faulty
        self.our_share = our_share
        self.verify = verify
        self.combine_and_parity = combine_and_parity
        self.master_verify = master_verify
        self.received = {}  # BTreeMap<N, SignatureShare>
        self.had_input = False
        self.terminated = False

    def handle_input(self):  # :90-97
        if not self.had_input:
            self.had_input = True
            return self._get_coin()
        return _step()

    def handle_message(self, sender, share):  # :100-111
        if not self.terminated:
            return self.handle_share(sender, share)
        return _step()

    def _get_coin(self):  # :138-147
        if self.our_id not in self.index:
            return self.try_output()
        return self.handle_share(self.our_id, self.our_share)

    def handle_share(self, sender, share):  # :149-161
        if sender in self.index:
            if not self.verify(sender, share):
                return _step(faults=[(sender, "UnverifiedSignatureShareSender")])
            self.received[sender] = share
        else:
            return _step(error="UnknownSender")
        return self.try_output()

    def try_output(self):  # :163-181
        if self.had_input and len(self.received) > self.f:
            items = [(self.index[i], self.received[i]) for i in sorted(self.received)]
            try:
                sig, parity = self.combine_and_parity(items)
            except Exception as e:  # crypto error -> CombineAndVerifySigCrypto
                return _step(error="CombineAndVerifySigCrypto:%s" % e)
            if not self.master_verify(sig):
                return _step(error="VerificationFailed")
            self.terminated = True
            self.handle_input()
            return _step(output=parity)
        return _step()

    def run(self, events):
        out = []
        for ev in events:
            out.append(self.handle_input() if ev[0] == "input" else self.handle_message(ev[1], ev[2]))
        return out


class ThresholdDecryption:
    """threshold_decryption.rs:45 — verify(sender, share, ct), decrypt(items, ct) and
    ct_valid(ct) are injected; our_share(ct) is the share our node contributes."""

    def __init__(self, node_ids, our_id, num_faulty, our_share, verify, decrypt, ct_valid):
        self.ids = sorted(node_ids)
        self.index = {n: i for i, n in enumerate(self.ids)}
        self.our_id = our_id
        self.f = num_faulty
        self.our_share = our_share
        self.verify = verify
        self.decrypt = decrypt
        self.ct_valid = ct_valid
        self.ct = None
        self.shares = {}
        self.terminated = False

    def set_ciphertext(self, ct):  # :94-113
        if self.ct is not None:
            return _step(error="MultipleInputs")
        if not self.ct_valid(ct):
            return _step(error="InvalidCiphertext")
        self.ct = ct
        step = _step(faults=self._remove_invalid_shares())
        if self.our_id in self.index:
            self.shares[self.our_id] = self.our_share
        r = self.try_output()
        step["faults"] += r["faults"]
        step["output"], step["error"] = r["output"], r["error"]
        return step

    def handle_message(self, sender, share):  # :120-133
        if self.terminated:
            return _step()
        if not self._is_share_valid(sender, share):
            return _step(faults=[(sender, "UnverifiedDecryptionShareSender")])
        dup = sender in self.shares
        self.shares[sender] = share
        if dup:
            return _step(faults=[(sender, "MultipleDecryptionShares")])
        return self.try_output()

    def _remove_invalid_shares(self):  # :136-149
        bad = [i for i in sorted(self.shares) if not self._is_share_valid(i, self.shares[i])]
        for i in bad:
            del self.shares[i]
        return [(i, "UnverifiedDecryptionShareSender") for i in bad]

    def _is_share_valid(self, sender, share):  # :152-161
        if self.ct is None:
            return True
        if sender not in self.index:
            return False
        return self.verify(sender, share, self.ct)

    def try_output(self):  # :164-188
        if self.terminated or len(self.shares) <= self.f:
            return _step()
        if self.ct is None:
            return _step()
        self.terminated = True
        items = [(self.index[i], self.shares[i]) for i in sorted(self.shares)]
        try:
            return _step(output=self.decrypt(items, self.ct))
        except Exception as e:
            return _step(error="Decryption:%s" % e)

    def run(self, events):
        out = []
        for ev in events:
            out.append(self.set_ciphertext(ev[1]) if ev[0] == "ct" else self.handle_message(ev[1], ev[2]))
        return out


# ------------------------------------------------------------------------------ SyncKeyGen
def _fr_from_wire(b, pos=0):
    """bincode FieldWrap<Fr>: u64 LE length 32 + 32-byte big-endian value < r (restated)."""
    R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    if len(b) < pos + 40 or int.from_bytes(b[pos:pos + 8], "little") != 32:
        raise ValueError("FieldWrap")
    v = int.from_bytes(b[pos + 8:pos + 40], "big")
    if v >= R:
        raise ValueError("FieldWrap >= r")
    return v, pos + 40


def _poly_from_wire(b):
    if len(b) < 8:
        raise ValueError("Poly")
    n = int.from_bytes(b[:8], "little")
    if 8 + 40 * n > len(b):  # bincode 1.0 ignores bytes after the last field
        raise ValueError("Poly length")
    out, pos = [], 8
    for _ in range(n):
        v, pos = _fr_from_wire(b, pos)
        out.append(v)
    return out


class SyncKeyGen:
    """sync_key_gen.rs:272-509 — one node, every message handled the moment it arrives.
    Injected: decrypt(ct) -> bytes or None (SecretKey::decrypt), row_matches(commit, row) ->
    bool (row.commitment() == commit.row(our_idx + 1)), value_matches(commit, sender_idx, val)
    -> bool (commit.evaluate(our_idx + 1, sender_idx + 1) == val * G1)."""

    def __init__(self, node_ids, our_id, threshold, decrypt, row_matches, value_matches):
        self.ids = sorted(node_ids)
        self.index = {n: i for i, n in enumerate(self.ids)}
        self.our_idx = self.index.get(our_id)
        self.t = threshold
        self.decrypt = decrypt
        self.row_matches = row_matches
        self.value_matches = value_matches
        self.parts = {}  # sender_idx -> {"commit", "values", "acks"}

    def handle_part(self, sender, part):  # :338-381; part = (commit, rows)
        if sender not in self.index:
            return None
        s_idx = self.index[sender]
        commit, rows = part
        if s_idx in self.parts:
            return None
        self.parts[s_idx] = {"commit": commit, "values": {}, "acks": set()}
        if self.our_idx is None:
            return None
        if self.our_idx >= len(rows):
            return None
        ser_row = self.decrypt(rows[self.our_idx])
        if ser_row is None:
            return None
        try:
            row = _poly_from_wire(ser_row)
        except ValueError:
            return ("invalid", [(sender, "InvalidPartMessage")])
        if len(row) != self.t + 1 or not self.row_matches(commit, row):
            return ("invalid", [(sender, "InvalidPartMessage")])
        return ("valid", row)

    def handle_ack(self, sender, ack):  # :387-396 -> :462-498; ack = (proposer, values)
        if sender not in self.index:
            return []
        s_idx = self.index[sender]
        proposer, values = ack
        fault = lambda k: [(sender, ("AckMessage", k))]  # noqa: E731
        if len(values) != len(self.ids):
            return fault("NodeCount")
        part = self.parts.get(proposer)
        if part is None:
            return fault("SenderExist")
        if s_idx in part["acks"]:
            return fault("DuplicateAck")
        part["acks"].add(s_idx)
        if self.our_idx is None:
            return []
        ser_val = self.decrypt(values[self.our_idx])
        if ser_val is None:
            return fault("ValueDecryption")
        try:
            val, _ = _fr_from_wire(ser_val)  # trailing bytes ignored, as bincode 1.0 does
        except ValueError:
            return fault("ValueDeserialization")
        if not self.value_matches(part["commit"], s_idx, val):
            return fault("ValueInvalid")
        part["values"][s_idx + 1] = val
        return []

    def complete(self):
        return [p for p in sorted(self.parts) if len(self.parts[p]["acks"]) > 2 * self.t]

    def is_ready(self):
        return len(self.complete()) > self.t

    def secret_share(self):  # :428-447, the Fr half of generate()
        R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
        if self.our_idx is None:
            return None
        sk = 0
        for p in self.complete():
            items = sorted(self.parts[p]["values"].items())[:self.t + 1]
            for x, y in items:
                num = den = 1
                for x0, _ in items:
                    if x0 != x:
                        num = num * x0 % R
                        den = den * (x0 - x) % R
                sk = (sk + y * num * pow(den, R - 2, R)) % R
        return sk
