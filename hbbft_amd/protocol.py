"""Batch queues for hbbft's crypto call sites — the host-side mirror of the reference's Coin and
ThresholdDecryption decision logic, driving the GPU verifier.

The reference verifies every share synchronously on arrival (src/coin.rs:149-161,
src/threshold_decryption.rs:120-161).  Here every instance of an epoch queues its events; one
``flush`` verifies all queued shares of all instances in ONE batched GPU call, then REPLAYS each
instance's queue in arrival order with those verdicts.  Verdicts depend only on (sender, share,
nonce/ciphertext), never on protocol state, so the replay produces exactly the reference's faults,
errors and outputs; shares that arrive after termination are verified needlessly but, as in the
reference (coin.rs:105, td.rs:121-123), produce nothing.  Combines triggered during the replay
(try_output) are batched too; an instance whose deferred combine fails is replayed again in
synchronous mode so the reference's retry-on-error behaviour is kept.

Inputs are hbbft's wire encodings (compressed points).  H = hash_g2(nonce) / hash_g1_g2(u, v)
is supplied by the caller (threshold_crypto on the Rust side, per the design), and so is this
node's own share (signing is producer-side).  ThresholdDecryption outputs the combined point
g = sum l_i d_i (compressed); plaintext = v XOR hash_bytes(g, |v|) stays with the caller.
"""
from . import _native as N


def _step(faults=None, output=None, error=None):
    return {"faults": list(faults or []), "output": output, "error": error}


class NetInfo:
    """The parts of NetworkInfo (src/messaging.rs:222-269) the hot path reads."""

    def __init__(self, node_ids, our_id, keyset_id, master_pk=None):
        self.ids = sorted(node_ids)
        self.index = {n: i for i, n in enumerate(self.ids)}
        self.our_id = our_id
        self.num_faulty = (len(self.ids) - 1) // 3  # messaging.rs:260
        self.keyset = keyset_id
        self.master_pk = master_pk

    def is_validator(self):
        return self.our_id in self.index


# ================================================================================== Coin
class _CoinState:
    def __init__(self, H, our_share):
        self.H = H
        self.our_share = our_share
        self.events = []
        self.received = {}
        self.had_input = False
        self.terminated = False


class CoinEpoch:
    """Every Coin instance (coin.rs:64) of one epoch behind one batch queue."""

    def __init__(self, ctx, netinfo):
        self.ctx = ctx
        self.ni = netinfo
        self.inst = {}

    def add(self, key, H_c96, our_share_c96=None):
        self.inst[key] = _CoinState(bytes(H_c96), our_share_c96)

    def handle_input(self, key):
        self.inst[key].events.append(("input",))

    def handle_message(self, key, sender, share_c96):
        self.inst[key].events.append(("msg", sender, bytes(share_c96)))

    # ---------------------------------------------------------------- flush
    def flush(self):
        """Verify every queued share in one GPU call, replay, batch the combines.  Returns
        {key: [step per queued event]}."""
        ni = self.ni
        keys = [k for k in self.inst if self.inst[k].events]
        # state at the start of the flush: a failed deferred combine replays from here
        snap = {k: (dict(self.inst[k].received), self.inst[k].had_input, self.inst[k].terminated)
                for k in keys}
        counts, idx, sigs, where = [], [], [], {}
        for k in keys:
            st = self.inst[k]
            c = 0
            if st.terminated:  # coin.rs:105: nothing after termination is looked at
                counts.append(0)
                continue
            for e_i, ev in enumerate(st.events):
                share = None
                sender = None
                if ev[0] == "input" and ni.is_validator() and st.our_share is not None:
                    sender, share = ni.our_id, st.our_share
                elif ev[0] == "msg":
                    sender, share = ev[1], ev[2]
                if share is not None and sender in ni.index:
                    where[(k, e_i)] = len(idx)
                    idx.append(ni.index[sender])
                    sigs.append(share)
                    c += 1
            counts.append(c)
        verdict = {}
        if idx:
            status = self.ctx.verify_sig_shares(ni.keyset, [self.inst[k].H for k in keys], counts,
                                                idx, sigs)
            for key_ev, pos in where.items():
                verdict[key_ev] = int(status[pos]) == N.ACCEPT
        results, pending = {}, []
        for k in keys:
            results[k] = self._replay(k, verdict, pending)
        self._finish_combines(pending, results, verdict, snap)
        for k in keys:
            self.inst[k].events = []
        return results

    def _replay(self, k, verdict, pending, sync=False):
        st, ni = self.inst[k], self.ni
        steps = []
        for e_i, ev in enumerate(st.events):
            if ev[0] == "input":
                if st.had_input:
                    steps.append(_step())
                    continue
                st.had_input = True
                if not ni.is_validator():
                    steps.append(self._try_output(k, e_i, pending, sync))
                else:
                    steps.append(self._handle_share(k, e_i, ni.our_id, verdict, pending, sync))
            else:
                if st.terminated:
                    steps.append(_step())
                else:
                    steps.append(self._handle_share(k, e_i, ev[1], verdict, pending, sync))
        return steps

    def _handle_share(self, k, e_i, sender, verdict, pending, sync):  # coin.rs:149-161
        st, ni = self.inst[k], self.ni
        if sender not in ni.index:
            return _step(error="UnknownSender")
        if not verdict.get((k, e_i), False):
            return _step(faults=[(sender, "UnverifiedSignatureShareSender")])
        ev = st.events[e_i]
        st.received[sender] = ev[2] if ev[0] == "msg" else st.our_share
        return self._try_output(k, e_i, pending, sync)

    def _try_output(self, k, e_i, pending, sync):  # coin.rs:163-181
        st, ni = self.inst[k], self.ni
        if st.had_input and len(st.received) > ni.num_faulty:
            items = [(ni.index[i], st.received[i]) for i in sorted(st.received)]
            step = _step()
            if sync:
                res = self._combine([k], [items])[0]
                if res[0] is not None:
                    step["error"] = res[0]
                    return step
                step["output"] = res[1]
            else:
                pending.append((k, e_i, items, step))
            st.terminated = True
            return step
        return _step()

    def _combine(self, keys, item_lists):
        """[(error-or-None, parity)] via one hbtc_combine_sigs + one hbtc_verify_sigs call
        (the master-key check of coin.rs:192-197)."""
        t = self.ni.num_faulty + 1
        counts = [len(it) for it in item_lists]
        idx = [i for it in item_lists for i, _ in it]
        sigs = [s for it in item_lists for _, s in it]
        out, par, cst = self.ctx.combine_sigs(counts, idx, sigs, t)
        res = [None] * len(item_lists)
        ok_pos = [j for j in range(len(item_lists)) if int(cst[j]) == N.ACCEPT]
        for j in range(len(item_lists)):
            if int(cst[j]) != N.ACCEPT:
                res[j] = ("CombineAndVerifySigCrypto:%s" % N.STATUS_NAMES[int(cst[j])], None)
        if ok_pos and self.ni.master_pk is not None:
            Hs = [self.inst[keys[j]].H for j in ok_pos]
            vs = self.ctx.verify_sigs([self.ni.master_pk] * len(ok_pos), Hs, [out[j] for j in ok_pos])
            for j, v in zip(ok_pos, vs):
                res[j] = (None, bool(par[j])) if int(v) == N.ACCEPT else ("VerificationFailed", None)
        else:
            for j in ok_pos:
                res[j] = (None, bool(par[j]))
        return res

    def _finish_combines(self, pending, results, verdict, snap):
        if not pending:
            return
        res = self._combine([p[0] for p in pending], [p[2] for p in pending])
        failed = set()
        for (k, e_i, items, step), (err, parity) in zip(pending, res):
            if err is None:
                step["output"] = parity
            else:
                failed.add(k)
        for k in failed:  # rare: redo this flush of the instance with synchronous combines,
            st = self.inst[k]  # from its state at the start of the flush (coin.rs:163-181 retries)
            received, had_input, terminated = snap[k]
            st.received, st.had_input, st.terminated = dict(received), had_input, terminated
            results[k] = self._replay(k, verdict, [], sync=True)


# ================================================================================== ThresholdDecryption
class _TdState:
    def __init__(self, our_share):
        self.our_share = our_share
        self.events = []
        self.ct = None  # (u_c48, v, w_c96, H_c96)
        self.shares = {}
        self.terminated = False


class DecryptionEpoch:
    """Every ThresholdDecryption instance (threshold_decryption.rs:45) of one epoch."""

    def __init__(self, ctx, netinfo):
        self.ctx = ctx
        self.ni = netinfo
        self.inst = {}

    def add(self, key, our_share_c48=None):
        self.inst[key] = _TdState(our_share_c48)

    def set_ciphertext(self, key, u_c48, v, w_c96, H_c96):
        self.inst[key].events.append(("ct", (bytes(u_c48), bytes(v), bytes(w_c96), bytes(H_c96))))

    def handle_message(self, key, sender, share_c48):
        self.inst[key].events.append(("msg", sender, bytes(share_c48)))

    def flush(self):
        ni = self.ni
        keys = [k for k in self.inst if self.inst[k].events]
        # every queued ciphertext of an instance that has none yet: set_ciphertext leaves the
        # instance without one after an invalid ciphertext (td.rs:94-105), so a later valid one
        # in the same queue is accepted
        ct_ev = []
        for k in keys:
            st = self.inst[k]
            if st.ct is None:
                ct_ev += [(k, e_i, ev[1]) for e_i, ev in enumerate(st.events) if ev[0] == "ct"]
        ct_ok = {}
        if ct_ev:
            vs = self.ctx.verify_ciphertexts([c[0] for _, _, c in ct_ev], [c[3] for _, _, c in ct_ev],
                                             [c[2] for _, _, c in ct_ev])
            for (k, e_i, _), v in zip(ct_ev, vs):
                ct_ok[(k, e_i)] = int(v) == N.ACCEPT
        # the ciphertext each instance will know by the end of its queue: the stored one, else
        # the first valid queued one
        ct_of = {}
        for k in keys:
            st = self.inst[k]
            ct = st.ct
            if ct is None:
                ct = next((ev[1] for e_i, ev in enumerate(st.events)
                           if ev[0] == "ct" and ct_ok.get((k, e_i), False)), None)
            ct_of[k] = ct
        # shares that will be checked against that ciphertext: the stored (still unverified)
        # ones when it is set in this flush (remove_invalid_shares, td.rs:136-149), and every
        # queued message of an instance that has not terminated (td.rs:121-128)
        vkeys, counts, idx, shares, where = [], [], [], [], {}
        for k in keys:
            st, ct = self.inst[k], ct_of[k]
            if ct is None or st.terminated:
                continue
            cand = [("stored", s, sh) for s, sh in st.shares.items()] if st.ct is None else []
            cand += [("ev%d" % e_i, ev[1], ev[2]) for e_i, ev in enumerate(st.events) if ev[0] == "msg"]
            c = 0
            for tag, sender, sh in cand:
                if sender in ni.index:
                    where[(k, tag, sender)] = len(idx)
                    idx.append(ni.index[sender])
                    shares.append(sh)
                    c += 1
            if c:
                vkeys.append(k)
                counts.append(c)
        verdict = {}
        if idx:
            status = self.ctx.verify_dec_shares(ni.keyset, [ct_of[k][3] for k in vkeys],
                                                [ct_of[k][2] for k in vkeys], counts, idx, shares)
            for key, pos in where.items():
                verdict[key] = int(status[pos]) == N.ACCEPT
        results, pending = {}, []
        for k in keys:
            results[k] = self._replay(k, verdict, ct_ok, pending)
        if pending:
            t = ni.num_faulty + 1
            g, cst = self.ctx.combine_dec([len(p[2]) for p in pending],
                                          [i for p in pending for i, _ in p[2]],
                                          [s for p in pending for _, s in p[2]], t)
            for (k, step, items), gk, c in zip(pending, g, cst):
                if int(c) == N.ACCEPT:
                    step["output"] = gk
                else:
                    step["error"] = "Decryption:%s" % N.STATUS_NAMES[int(c)]
        for k in keys:
            self.inst[k].events = []
            for step in results[k]:
                step.pop("_pending", None)
        return results

    def _valid(self, k, tag, sender, verdict):  # td.rs:152-161 (with the ciphertext known)
        if sender not in self.ni.index:
            return False
        return verdict.get((k, tag, sender), False)

    def _replay(self, k, verdict, ct_ok, pending):
        st, ni = self.inst[k], self.ni
        steps = []
        stored_tag = {s: "stored" for s in st.shares}
        for e_i, ev in enumerate(st.events):
            if ev[0] == "ct":  # set_ciphertext, td.rs:94-113
                if st.ct is not None:
                    steps.append(_step(error="MultipleInputs"))
                    continue
                if not ct_ok.get((k, e_i), False):
                    steps.append(_step(error="InvalidCiphertext"))
                    continue
                st.ct = ev[1]
                bad = [s for s in sorted(st.shares) if not self._valid(k, stored_tag[s], s, verdict)]
                for s in bad:
                    del st.shares[s]
                step = _step(faults=[(s, "UnverifiedDecryptionShareSender") for s in bad])
                if ni.is_validator():
                    st.shares[ni.our_id] = st.our_share
                    stored_tag[ni.our_id] = "own"
                r = self._try_output(k, pending)
                step["faults"] += r["faults"]
                step["output"] = r["output"]
                if r is not step and r.get("_pending"):
                    pending[-1] = (pending[-1][0], step, pending[-1][2])
                steps.append(step)
            else:  # handle_message, td.rs:120-133
                sender, share = ev[1], ev[2]
                if st.terminated:
                    steps.append(_step())
                    continue
                tag = "ev%d" % e_i
                if st.ct is not None and not self._valid(k, tag, sender, verdict):
                    steps.append(_step(faults=[(sender, "UnverifiedDecryptionShareSender")]))
                    continue
                dup = sender in st.shares
                st.shares[sender] = share
                stored_tag[sender] = tag
                if dup:
                    steps.append(_step(faults=[(sender, "MultipleDecryptionShares")]))
                    continue
                steps.append(self._try_output(k, pending))
        return steps

    def _try_output(self, k, pending):  # td.rs:164-188
        st, ni = self.inst[k], self.ni
        if st.terminated or len(st.shares) <= ni.num_faulty or st.ct is None:
            return _step()
        st.terminated = True
        items = [(ni.index[i], st.shares[i]) for i in sorted(st.shares)]
        step = _step()
        step["_pending"] = True
        pending.append((k, step, items))
        return step
