//! Per-epoch batch queues for hbbft's Coin and ThresholdDecryption call sites: the Rust form of
//! `hbbft_amd/protocol.py` (whose tests check it against a sequential restatement of the
//! reference's rules, `oracle/hbbft_rules.py`).  Written against this crate's safe layer; no
//! Rust toolchain exists in the build image, so this file is not compiled here.
//!
//! The reference verifies every share synchronously on arrival (`src/coin.rs:149-161`,
//! `src/threshold_decryption.rs:120-161`).  A queue records an epoch's events per instance;
//! `flush` verifies every queued share of every instance in ONE batched call, then replays each
//! instance's events in arrival order with those verdicts.  A verdict depends only on (sender,
//! share, nonce / ciphertext), never on protocol state, so the replay yields the reference's
//! faults, errors and outputs.  The combines that the replay triggers are batched as well; a Coin
//! instance whose deferred combine fails is replayed again with synchronous combines, which keeps
//! the reference's retry-on-error behaviour (`src/coin.rs:163-181`).
//!
//! H = hash_g2(nonce) / hash_g1_g2(u, v) is supplied by the caller (`hash_g2` of this crate, or
//! `hbtc_hash_*_batch_gpu` for a whole epoch), and so is this node's own share.

use std::collections::{BTreeMap, BTreeSet};

use crate::{Batch, Context, Result, ACCEPT};

/// The parts of NetworkInfo (`src/messaging.rs:222-269`) the hot path reads.
pub struct NetInfo<N: Ord + Clone> {
    index: BTreeMap<N, u32>,
    our_id: N,
    num_faulty: usize,
    keyset: u32,
    master_pk: Option<[u8; 48]>,
}

impl<N: Ord + Clone> NetInfo<N> {
    pub fn new(node_ids: &[N], our_id: N, keyset: u32, master_pk: Option<[u8; 48]>) -> Self {
        let ids: BTreeSet<N> = node_ids.iter().cloned().collect();
        let index = ids.iter().cloned().enumerate().map(|(i, n)| (n, i as u32)).collect();
        let num_faulty = (ids.len().max(1) - 1) / 3; // messaging.rs:260
        NetInfo { index, our_id, num_faulty, keyset, master_pk }
    }

    pub fn is_validator(&self) -> bool {
        self.index.contains_key(&self.our_id)
    }
}

#[derive(Debug, Clone, PartialEq, Eq)]
pub enum FaultKind {
    UnverifiedSignatureShareSender,
    UnverifiedDecryptionShareSender,
    MultipleDecryptionShares,
}

/// One replayed event's result, as the reference's `Step`: faults, an output or an error.
#[derive(Debug, Clone)]
pub struct Step<N, O> {
    pub faults: Vec<(N, FaultKind)>,
    pub output: Option<O>,
    pub error: Option<String>,
}

impl<N, O> Default for Step<N, O> {
    fn default() -> Self {
        Step { faults: Vec::new(), output: None, error: None }
    }
}

fn csr(counts: &[u32]) -> Vec<u32> {
    let mut off = Vec::with_capacity(counts.len() + 1);
    off.push(0u32);
    for c in counts {
        let last = *off.last().unwrap();
        off.push(last + c);
    }
    off
}

// ========================================================================================== Coin
enum CoinEvent<N> {
    Input,
    Msg(N, [u8; 96]),
}

struct CoinState<N> {
    h: [u8; 96],
    our_share: Option<[u8; 96]>,
    events: Vec<CoinEvent<N>>,
    received: BTreeMap<N, [u8; 96]>,
    had_input: bool,
    terminated: bool,
}

/// A combine the replay asked for: (instance, event, its step slot, the shares in node order).
struct PendingCoin<K> {
    key: K,
    event: usize,
    items: Vec<(u32, [u8; 96])>,
}

/// Every Coin instance (`src/coin.rs:64`) of one epoch behind one queue.  Output: the coin's
/// parity bit.
pub struct CoinEpoch<K: Ord + Clone, N: Ord + Clone> {
    ni: NetInfo<N>,
    inst: BTreeMap<K, CoinState<N>>,
}

impl<K: Ord + Clone, N: Ord + Clone> CoinEpoch<K, N> {
    pub fn new(ni: NetInfo<N>) -> Self {
        CoinEpoch { ni, inst: BTreeMap::new() }
    }

    pub fn add(&mut self, key: K, h_c96: [u8; 96], our_share_c96: Option<[u8; 96]>) {
        self.inst.insert(key, CoinState { h: h_c96, our_share: our_share_c96, events: Vec::new(),
                                          received: BTreeMap::new(), had_input: false, terminated: false });
    }

    pub fn handle_input(&mut self, key: &K) {
        self.inst.get_mut(key).expect("unknown coin").events.push(CoinEvent::Input);
    }

    pub fn handle_message(&mut self, key: &K, sender: N, share_c96: [u8; 96]) {
        self.inst.get_mut(key).expect("unknown coin").events.push(CoinEvent::Msg(sender, share_c96));
    }

    /// Verify every queued share in one call, replay, batch the combines.  Returns the steps of
    /// every queued event, per instance.
    pub fn flush(&mut self, ctx: &Context) -> Result<BTreeMap<K, Vec<Step<N, bool>>>> {
        let keys: Vec<K> = self.inst.iter().filter(|(_, s)| !s.events.is_empty()).map(|(k, _)| k.clone()).collect();
        // the state at the start of the flush: a failed deferred combine replays from here
        let snap: BTreeMap<K, (BTreeMap<N, [u8; 96]>, bool, bool)> = keys.iter()
            .map(|k| { let s = &self.inst[k]; (k.clone(), (s.received.clone(), s.had_input, s.terminated)) })
            .collect();
        let (mut counts, mut idx, mut sigs, mut hs) = (Vec::new(), Vec::new(), Vec::new(), Vec::new());
        let mut slot: BTreeMap<(K, usize), usize> = BTreeMap::new();
        for k in &keys {
            let st = &self.inst[k];
            hs.extend_from_slice(&st.h);
            let mut c = 0u32;
            if !st.terminated {  // coin.rs:105: nothing after termination is looked at
                for (e, ev) in st.events.iter().enumerate() {
                    let share = match ev {
                        CoinEvent::Input if self.ni.is_validator() => st.our_share.map(|s| (self.ni.our_id.clone(), s)),
                        CoinEvent::Input => None,
                        CoinEvent::Msg(sender, s) => Some((sender.clone(), *s)),
                    };
                    if let Some((sender, s)) = share {
                        if let Some(&i) = self.ni.index.get(&sender) {
                            slot.insert((k.clone(), e), idx.len());
                            idx.push(i);
                            sigs.extend_from_slice(&s);
                            c += 1;
                        }
                    }
                }
            }
            counts.push(c);
        }
        let mut verdict: BTreeMap<(K, usize), bool> = BTreeMap::new();
        if !idx.is_empty() {
            let offsets = csr(&counts);
            let status = ctx.verify_sig_shares(self.ni.keyset, &hs, &Batch { offsets: &offsets, idx: &idx, items: &sigs })?;
            for (key_ev, pos) in slot {
                verdict.insert(key_ev, status[pos] == ACCEPT);
            }
        }
        let mut results = BTreeMap::new();
        let mut pending = Vec::new();
        for k in &keys {
            let steps = self.replay(k, &verdict, &mut pending, None)?;
            results.insert(k.clone(), steps);
        }
        self.finish_combines(ctx, pending, &mut results, &verdict, snap)?;
        for k in &keys {
            self.inst.get_mut(k).unwrap().events.clear();
        }
        Ok(results)
    }

    /// Replays an instance's queue.  `sync`: combine right away (the retry path) instead of
    /// deferring to the batched combine.
    fn replay(&mut self, k: &K, verdict: &BTreeMap<(K, usize), bool>, pending: &mut Vec<PendingCoin<K>>,
              sync: Option<&Context>) -> Result<Vec<Step<N, bool>>> {
        let n_events = self.inst[k].events.len();
        let mut steps = Vec::with_capacity(n_events);
        for e in 0..n_events {
            let is_input = matches!(self.inst[k].events[e], CoinEvent::Input);
            let step = if is_input {
                let st = self.inst.get_mut(k).unwrap();
                if st.had_input {
                    Step::default()
                } else {
                    st.had_input = true;
                    if !self.ni.is_validator() {
                        self.try_output(k, e, pending, sync)?
                    } else {
                        let me = self.ni.our_id.clone();
                        self.handle_share(k, e, me, verdict, pending, sync)?
                    }
                }
            } else if self.inst[k].terminated {
                Step::default()
            } else {
                let sender = match &self.inst[k].events[e] { CoinEvent::Msg(s, _) => s.clone(), CoinEvent::Input => unreachable!() };
                self.handle_share(k, e, sender, verdict, pending, sync)?
            };
            steps.push(step);
        }
        Ok(steps)
    }

    // coin.rs:149-161
    fn handle_share(&mut self, k: &K, e: usize, sender: N, verdict: &BTreeMap<(K, usize), bool>,
                    pending: &mut Vec<PendingCoin<K>>, sync: Option<&Context>) -> Result<Step<N, bool>> {
        if !self.ni.index.contains_key(&sender) {
            return Ok(Step { error: Some("UnknownSender".into()), ..Step::default() });
        }
        if !verdict.get(&(k.clone(), e)).copied().unwrap_or(false) {
            return Ok(Step { faults: vec![(sender, FaultKind::UnverifiedSignatureShareSender)], ..Step::default() });
        }
        let st = self.inst.get_mut(k).unwrap();
        let share = match &st.events[e] { CoinEvent::Msg(_, s) => *s, CoinEvent::Input => st.our_share.unwrap() };
        st.received.insert(sender, share);
        self.try_output(k, e, pending, sync)
    }

    // coin.rs:163-181
    fn try_output(&mut self, k: &K, e: usize, pending: &mut Vec<PendingCoin<K>>, sync: Option<&Context>)
        -> Result<Step<N, bool>> {
        let num_faulty = self.ni.num_faulty;
        let st = &self.inst[k];
        if !(st.had_input && st.received.len() > num_faulty) {
            return Ok(Step::default());
        }
        let items: Vec<(u32, [u8; 96])> = st.received.iter().map(|(n, s)| (self.ni.index[n], *s)).collect();
        let mut step = Step::default();
        if let Some(ctx) = sync {
            match self.combine(ctx, &[k.clone()], &[items])?.remove(0) {
                Err(msg) => {
                    step.error = Some(msg);
                    return Ok(step);
                }
                Ok(parity) => step.output = Some(parity),
            }
        } else {
            pending.push(PendingCoin { key: k.clone(), event: e, items });
        }
        self.inst.get_mut(k).unwrap().terminated = true;
        Ok(step)
    }

    /// combine_signatures of the first t shares (node order) + the master-key check of
    /// coin.rs:192-197, for several instances in one call each.
    fn combine(&self, ctx: &Context, keys: &[K], lists: &[Vec<(u32, [u8; 96])>]) -> Result<Vec<std::result::Result<bool, String>>> {
        let t = (self.ni.num_faulty + 1) as u32;
        let counts: Vec<u32> = lists.iter().map(|l| l.len() as u32).collect();
        let offsets = csr(&counts);
        let idx: Vec<u32> = lists.iter().flat_map(|l| l.iter().map(|(i, _)| *i)).collect();
        let sigs: Vec<u8> = lists.iter().flat_map(|l| l.iter().flat_map(|(_, s)| s.iter().copied())).collect();
        let (out, par, cst) = ctx.combine_sigs(&Batch { offsets: &offsets, idx: &idx, items: &sigs }, t)?;
        let mut res: Vec<std::result::Result<bool, String>> =
            (0..lists.len()).map(|j| if cst[j] == ACCEPT { Ok(par[j] != 0) } else { Err(format!("CombineAndVerifySigCrypto:{}", cst[j])) }).collect();
        if let Some(mpk) = self.ni.master_pk {
            let ok: Vec<usize> = (0..lists.len()).filter(|&j| cst[j] == ACCEPT).collect();
            if !ok.is_empty() {
                let pks: Vec<u8> = ok.iter().flat_map(|_| mpk.iter().copied()).collect();
                let hs: Vec<u8> = ok.iter().flat_map(|&j| self.inst[&keys[j]].h.iter().copied()).collect();
                let ss: Vec<u8> = ok.iter().flat_map(|&j| out[96 * j..96 * j + 96].iter().copied()).collect();
                let vs = ctx.verify_sigs(&pks, &hs, &ss)?;
                for (j, v) in ok.into_iter().zip(vs) {
                    if v != ACCEPT {
                        res[j] = Err("VerificationFailed".into());
                    }
                }
            }
        }
        Ok(res)
    }

    fn finish_combines(&mut self, ctx: &Context, pending: Vec<PendingCoin<K>>,
                       results: &mut BTreeMap<K, Vec<Step<N, bool>>>, verdict: &BTreeMap<(K, usize), bool>,
                       snap: BTreeMap<K, (BTreeMap<N, [u8; 96]>, bool, bool)>) -> Result<()> {
        if pending.is_empty() {
            return Ok(());
        }
        let keys: Vec<K> = pending.iter().map(|p| p.key.clone()).collect();
        let lists: Vec<Vec<(u32, [u8; 96])>> = pending.iter().map(|p| p.items.clone()).collect();
        let res = self.combine(ctx, &keys, &lists)?;
        let mut failed = BTreeSet::new();
        for (p, r) in pending.iter().zip(res) {
            match r {
                Ok(parity) => results.get_mut(&p.key).unwrap()[p.event].output = Some(parity),
                Err(_) => { failed.insert(p.key.clone()); }
            }
        }
        // rare: redo this flush of the instance with synchronous combines, from its state at the
        // start of the flush (coin.rs:163-181 retries on error)
        for k in failed {
            let (received, had_input, terminated) = snap[&k].clone();
            {
                let st = self.inst.get_mut(&k).unwrap();
                st.received = received;
                st.had_input = had_input;
                st.terminated = terminated;
            }
            let mut none = Vec::new();
            let steps = self.replay(&k, verdict, &mut none, Some(ctx))?;
            results.insert(k, steps);
        }
        Ok(())
    }
}

// =========================================================================== ThresholdDecryption
/// A ciphertext as the queue needs it: u (G1), v, w (G2) and H = hash_g1_g2(u, v).
#[derive(Clone)]
pub struct Ct {
    pub u: [u8; 48],
    pub v: Vec<u8>,
    pub w: [u8; 96],
    pub h: [u8; 96],
}

enum TdEvent<N> {
    Ciphertext(Ct),
    Msg(N, [u8; 48]),
}

/// Where a stored share came from: verified at set_ciphertext time (Stored), our own, or event e.
#[derive(Clone, Copy, PartialEq, Eq, PartialOrd, Ord)]
enum Tag {
    Stored,
    Own,
    Event(usize),
}

struct TdState<N> {
    our_share: Option<[u8; 48]>,
    events: Vec<TdEvent<N>>,
    ct: Option<Ct>,
    shares: BTreeMap<N, [u8; 48]>,
    terminated: bool,
}

/// Every ThresholdDecryption instance (`src/threshold_decryption.rs:45`) of one epoch.  Output:
/// the combined point g = sum l_i d_i (compressed G1); plaintext = v ^ hash_bytes(g, |v|).
pub struct DecryptionEpoch<K: Ord + Clone, N: Ord + Clone> {
    ni: NetInfo<N>,
    inst: BTreeMap<K, TdState<N>>,
}

impl<K: Ord + Clone, N: Ord + Clone> DecryptionEpoch<K, N> {
    pub fn new(ni: NetInfo<N>) -> Self {
        DecryptionEpoch { ni, inst: BTreeMap::new() }
    }

    pub fn add(&mut self, key: K, our_share_c48: Option<[u8; 48]>) {
        self.inst.insert(key, TdState { our_share: our_share_c48, events: Vec::new(), ct: None,
                                        shares: BTreeMap::new(), terminated: false });
    }

    pub fn set_ciphertext(&mut self, key: &K, ct: Ct) {
        self.inst.get_mut(key).expect("unknown instance").events.push(TdEvent::Ciphertext(ct));
    }

    pub fn handle_message(&mut self, key: &K, sender: N, share_c48: [u8; 48]) {
        self.inst.get_mut(key).expect("unknown instance").events.push(TdEvent::Msg(sender, share_c48));
    }

    pub fn flush(&mut self, ctx: &Context) -> Result<BTreeMap<K, Vec<Step<N, [u8; 48]>>>> {
        let keys: Vec<K> = self.inst.iter().filter(|(_, s)| !s.events.is_empty()).map(|(k, _)| k.clone()).collect();
        // Ciphertext::verify of every queued ciphertext of an instance that has none yet
        // (set_ciphertext leaves it without one after an invalid ciphertext, td.rs:94-105)
        let mut ct_ev: Vec<(K, usize)> = Vec::new();
        let (mut us, mut hs, mut ws) = (Vec::new(), Vec::new(), Vec::new());
        for k in &keys {
            let st = &self.inst[k];
            if st.ct.is_none() {
                for (e, ev) in st.events.iter().enumerate() {
                    if let TdEvent::Ciphertext(c) = ev {
                        ct_ev.push((k.clone(), e));
                        us.extend_from_slice(&c.u);
                        hs.extend_from_slice(&c.h);
                        ws.extend_from_slice(&c.w);
                    }
                }
            }
        }
        let mut ct_ok: BTreeMap<(K, usize), bool> = BTreeMap::new();
        if !ct_ev.is_empty() {
            let vs = ctx.verify_ciphertexts(&us, &hs, &ws)?;
            for (ke, v) in ct_ev.into_iter().zip(vs) {
                ct_ok.insert(ke, v == ACCEPT);
            }
        }
        // the ciphertext each instance knows by the end of its queue
        let mut ct_of: BTreeMap<K, Option<Ct>> = BTreeMap::new();
        for k in &keys {
            let st = &self.inst[k];
            let ct = st.ct.clone().or_else(|| st.events.iter().enumerate().find_map(|(e, ev)| match ev {
                TdEvent::Ciphertext(c) if ct_ok.get(&(k.clone(), e)).copied().unwrap_or(false) => Some(c.clone()),
                _ => None,
            }));
            ct_of.insert(k.clone(), ct);
        }
        // the shares checked against it: the stored (unverified) ones when it is set in this flush
        // (remove_invalid_shares, td.rs:136-149) and every queued message (td.rs:121-128)
        let (mut counts, mut idx, mut items, mut vh, mut vw) = (Vec::new(), Vec::new(), Vec::new(), Vec::new(), Vec::new());
        let mut slot: BTreeMap<(K, Tag, N), usize> = BTreeMap::new();
        for k in &keys {
            let st = &self.inst[k];
            let ct = match (&ct_of[k], st.terminated) { (Some(c), false) => c, _ => continue };
            let mut cand: Vec<(Tag, N, [u8; 48])> = Vec::new();
            if st.ct.is_none() {
                cand.extend(st.shares.iter().map(|(s, sh)| (Tag::Stored, s.clone(), *sh)));
            }
            for (e, ev) in st.events.iter().enumerate() {
                if let TdEvent::Msg(s, sh) = ev {
                    cand.push((Tag::Event(e), s.clone(), *sh));
                }
            }
            let mut c = 0u32;
            for (tag, sender, sh) in cand {
                if let Some(&i) = self.ni.index.get(&sender) {
                    slot.insert((k.clone(), tag, sender), idx.len());
                    idx.push(i);
                    items.extend_from_slice(&sh);
                    c += 1;
                }
            }
            if c > 0 {
                counts.push(c);
                vh.extend_from_slice(&ct.h);
                vw.extend_from_slice(&ct.w);
            }
        }
        let mut verdict: BTreeMap<(K, Tag, N), bool> = BTreeMap::new();
        if !idx.is_empty() {
            let offsets = csr(&counts);
            let status = ctx.verify_dec_shares(self.ni.keyset, &vh, &vw, &Batch { offsets: &offsets, idx: &idx, items: &items })?;
            for (key, pos) in slot {
                verdict.insert(key, status[pos] == ACCEPT);
            }
        }
        let mut results = BTreeMap::new();
        let mut pending: Vec<(K, usize, Vec<(u32, [u8; 48])>)> = Vec::new();
        for k in &keys {
            let steps = self.replay(k, &verdict, &ct_ok, &mut pending);
            results.insert(k.clone(), steps);
        }
        if !pending.is_empty() {
            let t = (self.ni.num_faulty + 1) as u32;
            let counts: Vec<u32> = pending.iter().map(|p| p.2.len() as u32).collect();
            let offsets = csr(&counts);
            let idx: Vec<u32> = pending.iter().flat_map(|p| p.2.iter().map(|(i, _)| *i)).collect();
            let sh: Vec<u8> = pending.iter().flat_map(|p| p.2.iter().flat_map(|(_, s)| s.iter().copied())).collect();
            let (g, cst) = ctx.combine_dec(&Batch { offsets: &offsets, idx: &idx, items: &sh }, t)?;
            for (j, (k, e, _)) in pending.into_iter().enumerate() {
                let step: &mut Step<N, [u8; 48]> = &mut results.get_mut(&k).unwrap()[e];
                if cst[j] == ACCEPT {
                    let mut out = [0u8; 48];
                    out.copy_from_slice(&g[48 * j..48 * j + 48]);
                    step.output = Some(out);
                } else {
                    step.error = Some(format!("Decryption:{}", cst[j]));
                }
            }
        }
        for k in &keys {
            self.inst.get_mut(k).unwrap().events.clear();
        }
        Ok(results)
    }

    fn valid(&self, k: &K, tag: Tag, sender: &N, verdict: &BTreeMap<(K, Tag, N), bool>) -> bool {
        self.ni.index.contains_key(sender) && verdict.get(&(k.clone(), tag, sender.clone())).copied().unwrap_or(false)
    }

    fn replay(&mut self, k: &K, verdict: &BTreeMap<(K, Tag, N), bool>, ct_ok: &BTreeMap<(K, usize), bool>,
              pending: &mut Vec<(K, usize, Vec<(u32, [u8; 48])>)>) -> Vec<Step<N, [u8; 48]>> {
        let n_events = self.inst[k].events.len();
        let mut stored_tag: BTreeMap<N, Tag> = self.inst[k].shares.keys().map(|s| (s.clone(), Tag::Stored)).collect();
        let mut steps = Vec::with_capacity(n_events);
        for e in 0..n_events {
            let ct = match &self.inst[k].events[e] { TdEvent::Ciphertext(c) => Some(c.clone()), TdEvent::Msg(..) => None };
            if let Some(ct) = ct {  // set_ciphertext, td.rs:94-113
                if self.inst[k].ct.is_some() {
                    steps.push(Step { error: Some("MultipleInputs".into()), ..Step::default() });
                    continue;
                }
                if !ct_ok.get(&(k.clone(), e)).copied().unwrap_or(false) {
                    steps.push(Step { error: Some("InvalidCiphertext".into()), ..Step::default() });
                    continue;
                }
                let senders: Vec<N> = self.inst[k].shares.keys().cloned().collect();
                let bad: Vec<N> = senders.into_iter().filter(|s| !self.valid(k, stored_tag[s], s, verdict)).collect();
                let mut step = Step::default();
                {
                    let st = self.inst.get_mut(k).unwrap();
                    st.ct = Some(ct);
                    for s in &bad {
                        st.shares.remove(s);
                    }
                }
                step.faults = bad.into_iter().map(|s| (s, FaultKind::UnverifiedDecryptionShareSender)).collect();
                if self.ni.is_validator() {
                    let me = self.ni.our_id.clone();
                    let st = self.inst.get_mut(k).unwrap();
                    if let Some(own) = st.our_share {
                        st.shares.insert(me.clone(), own);
                    }
                    stored_tag.insert(me, Tag::Own);
                }
                self.try_output(k, e, pending);
                steps.push(step);
            } else {  // handle_message, td.rs:120-133
                let (sender, share) = match &self.inst[k].events[e] { TdEvent::Msg(s, sh) => (s.clone(), *sh), _ => unreachable!() };
                if self.inst[k].terminated {
                    steps.push(Step::default());
                    continue;
                }
                let tag = Tag::Event(e);
                if self.inst[k].ct.is_some() && !self.valid(k, tag, &sender, verdict) {
                    steps.push(Step { faults: vec![(sender, FaultKind::UnverifiedDecryptionShareSender)], ..Step::default() });
                    continue;
                }
                let dup = {
                    let st = self.inst.get_mut(k).unwrap();
                    st.shares.insert(sender.clone(), share).is_some()
                };
                stored_tag.insert(sender.clone(), tag);
                if dup {
                    steps.push(Step { faults: vec![(sender, FaultKind::MultipleDecryptionShares)], ..Step::default() });
                    continue;
                }
                self.try_output(k, e, pending);
                steps.push(Step::default());
            }
        }
        steps
    }

    // td.rs:164-188: the combine is deferred to the flush's batched call (output set there)
    fn try_output(&mut self, k: &K, e: usize, pending: &mut Vec<(K, usize, Vec<(u32, [u8; 48])>)>) {
        let num_faulty = self.ni.num_faulty;
        let st = &self.inst[k];
        if st.terminated || st.shares.len() <= num_faulty || st.ct.is_none() {
            return;
        }
        let items: Vec<(u32, [u8; 48])> = st.shares.iter().map(|(n, s)| (self.ni.index[n], *s)).collect();
        self.inst.get_mut(k).unwrap().terminated = true;
        pending.push((k.clone(), e, items));
    }
}

// ===================================================================================== SyncKeyGen
/// A threshold_crypto Ciphertext (u, v, w) as it arrives.
#[derive(Clone)]
pub struct WireCt {
    pub u: [u8; 48],
    pub v: Vec<u8>,
    pub w: [u8; 96],
}

/// The bincode decoding the replay needs (threshold_crypto's serde, provided by the caller):
/// a Part row -> t + 1 Fr (32-byte LE), an Ack value -> one Fr; None where serde refuses it.
pub trait SkgCodec {
    fn row(&self, plain: &[u8]) -> Option<Vec<[u8; 32]>>;
    fn value(&self, plain: &[u8]) -> Option<[u8; 32]>;
}

pub enum SkgMsg<N> {
    Part { sender: N, commit_c48: Vec<u8>, rows: Vec<WireCt> },
    Ack { sender: N, proposer: u32, values: Vec<WireCt> },
}

/// The outcome of one queued message (sync_key_gen.rs:338-398): a Part is ignored (None), valid
/// (our Ack is then built by the caller from `row`) or faulty; an Ack yields its faults.
pub enum SkgOutcome<N> {
    PartIgnored,
    PartValid { proposer: u32, row: Vec<[u8; 32]> },
    PartInvalid(N),
    Ack(Vec<(N, &'static str)>),
}

struct Proposal {
    commit: Vec<u8>,
    acks: BTreeSet<u32>,
    values: BTreeMap<u32, [u8; 32]>,
    our_row: Option<Vec<[u8; 32]>>,
}

/// One node's SyncKeyGen message handling with batched crypto (the Rust form of
/// `hbbft_amd/skg.py`): decrypt every queued ciphertext addressed to us in one `decrypt` call,
/// check every decoded row in one `skg_check_parts` call and every decoded value in one
/// `skg_check_acks` call against the commitment of the FIRST Part of its proposer (the only one
/// the reference stores, :346-354), then replay in order with the reference's fault order
/// NodeCount -> SenderExist -> DuplicateAck -> ValueDecryption -> ValueDeserialization ->
/// ValueInvalid (:467-495).
pub struct SkgQueue<N: Ord + Clone> {
    index: BTreeMap<N, u32>,
    our_idx: Option<u32>,
    sec_key_le32: [u8; 32],
    t: u32,
    parts: BTreeMap<u32, Proposal>,
    queue: Vec<SkgMsg<N>>,
}

impl<N: Ord + Clone> SkgQueue<N> {
    pub fn new(node_ids: &[N], our_id: &N, sec_key_le32: [u8; 32], t: u32) -> Self {
        let ids: BTreeSet<N> = node_ids.iter().cloned().collect();
        let index: BTreeMap<N, u32> = ids.iter().cloned().enumerate().map(|(i, n)| (n, i as u32)).collect();
        let our_idx = index.get(our_id).copied();
        SkgQueue { index, our_idx, sec_key_le32, t, parts: BTreeMap::new(), queue: Vec::new() }
    }

    pub fn handle(&mut self, msg: SkgMsg<N>) {
        self.queue.push(msg);
    }

    /// Ack values received so far for proposer p (node index + 1 -> Fr), for `generate`.
    pub fn values(&self, p: u32) -> Option<&BTreeMap<u32, [u8; 32]>> {
        self.parts.get(&p).map(|s| &s.values)
    }

    pub fn is_complete(&self, p: u32) -> bool {
        self.parts.get(&p).map_or(false, |s| s.acks.len() > 2 * self.t as usize)
    }

    pub fn flush(&mut self, ctx: &Context, codec: &dyn SkgCodec) -> Result<Vec<SkgOutcome<N>>> {
        let q = std::mem::take(&mut self.queue);
        let n = self.index.len();
        let t = self.t;
        // 1. the ciphertexts addressed to us, decrypted in one batch
        let mut jobs: Vec<usize> = Vec::new();
        let (mut us, mut ws, mut vs, mut off) = (Vec::new(), Vec::new(), Vec::new(), vec![0u32]);
        if let Some(our) = self.our_idx {
            for (m, msg) in q.iter().enumerate() {
                let (sender, cts, is_ack) = match msg {
                    SkgMsg::Part { sender, rows, .. } => (sender, rows, false),
                    SkgMsg::Ack { sender, values, .. } => (sender, values, true),
                };
                if !self.index.contains_key(sender) || (is_ack && cts.len() != n) {
                    continue;
                }
                if let Some(c) = cts.get(our as usize) {
                    jobs.push(m);
                    us.extend_from_slice(&c.u);
                    ws.extend_from_slice(&c.w);
                    vs.extend_from_slice(&c.v);
                    off.push(vs.len() as u32);
                }
            }
        }
        let mut plain: BTreeMap<usize, Option<Vec<u8>>> = BTreeMap::new();
        if !jobs.is_empty() {
            let (out, st) = ctx.decrypt(&self.sec_key_le32, &us, &ws, &vs, &off)?;
            for (j, m) in jobs.iter().enumerate() {
                let p = if st[j] == ACCEPT { Some(out[off[j] as usize..off[j + 1] as usize].to_vec()) } else { None };
                plain.insert(*m, p);
            }
        }
        // 2. decode; the commitment every message is checked against (first Part per proposer)
        let mut first: BTreeMap<u32, Vec<u8>> = self.parts.iter().map(|(p, s)| (*p, s.commit.clone())).collect();
        let mut commit_of: BTreeMap<usize, u32> = BTreeMap::new();  // message -> proposer whose commitment applies
        let mut rows: BTreeMap<usize, Option<Vec<[u8; 32]>>> = BTreeMap::new();
        let mut vals: BTreeMap<usize, Option<[u8; 32]>> = BTreeMap::new();
        for (m, msg) in q.iter().enumerate() {
            match msg {
                SkgMsg::Part { sender, commit_c48, .. } => {
                    let s = match self.index.get(sender) { Some(&s) => s, None => continue };
                    if !first.contains_key(&s) {
                        first.insert(s, commit_c48.clone());
                        commit_of.insert(m, s);
                    }
                    if let Some(Some(p)) = plain.get(&m) {
                        rows.insert(m, codec.row(p).filter(|r| r.len() == t as usize + 1));
                    }
                }
                SkgMsg::Ack { sender, proposer, .. } => {
                    if !self.index.contains_key(sender) {
                        continue;
                    }
                    if let Some(Some(p)) = plain.get(&m) {
                        vals.insert(m, codec.value(p));
                    }
                    if first.contains_key(proposer) {
                        commit_of.insert(m, *proposer);
                    }
                }
            }
        }
        // 3. batched checks
        let our = self.our_idx.unwrap_or(0);
        let mut row_ok: BTreeMap<usize, bool> = BTreeMap::new();
        let pm: Vec<usize> = rows.iter().filter(|(m, r)| r.is_some() && commit_of.contains_key(m)).map(|(m, _)| *m).collect();
        if !pm.is_empty() {
            let cm: Vec<u8> = pm.iter().flat_map(|m| first[&commit_of[m]].iter().copied()).collect();
            let rb: Vec<u8> = pm.iter().flat_map(|m| rows[m].as_ref().unwrap().iter().flat_map(|c| c.iter().copied())).collect();
            let st = ctx.skg_check_parts(t, our, &cm, &rb)?;
            for (m, s) in pm.iter().zip(st) {
                row_ok.insert(*m, s == ACCEPT);
            }
        }
        let mut val_ok: BTreeMap<usize, bool> = BTreeMap::new();
        let am: Vec<usize> = vals.iter().filter(|(m, v)| v.is_some() && commit_of.contains_key(m)).map(|(m, _)| *m).collect();
        if !am.is_empty() {
            // one commitment per distinct proposer, with our verified row when we have one
            let props: Vec<u32> = am.iter().map(|m| commit_of[m]).collect::<BTreeSet<_>>().into_iter().collect();
            let pos: BTreeMap<u32, u32> = props.iter().enumerate().map(|(i, p)| (*p, i as u32)).collect();
            let zero_row = vec![[0u8; 32]; t as usize + 1];
            let (mut cm, mut rb, mut ok) = (Vec::new(), Vec::new(), Vec::new());
            for p in &props {
                cm.extend_from_slice(&first[p]);
                let row = self.parts.get(p).and_then(|s| s.our_row.clone()).or_else(|| {
                    pm.iter().find(|m| commit_of[*m] == *p && row_ok.get(*m).copied().unwrap_or(false))
                        .and_then(|m| rows[m].clone())
                });
                ok.push(row.is_some() as u8);
                for c in row.as_ref().unwrap_or(&zero_row) {
                    rb.extend_from_slice(c);
                }
            }
            let ack_part: Vec<u32> = am.iter().map(|m| pos[&commit_of[m]]).collect();
            let ack_sender: Vec<u32> = am.iter().map(|m| match &q[*m] {
                SkgMsg::Ack { sender, .. } => self.index[sender],
                SkgMsg::Part { .. } => unreachable!(),
            }).collect();
            let vb: Vec<u8> = am.iter().flat_map(|m| vals[m].unwrap().to_vec()).collect();
            let st = ctx.skg_check_acks(t, our, &cm, &rb, &ok, &ack_part, &ack_sender, &vb)?;
            for (m, s) in am.iter().zip(st) {
                val_ok.insert(*m, s == ACCEPT);
            }
        }
        // 4. replay in order (:338-381 Parts, :387-396 / :462-498 Acks)
        let mut out = Vec::with_capacity(q.len());
        for (m, msg) in q.into_iter().enumerate() {
            let outcome = match msg {
                SkgMsg::Part { sender, commit_c48, rows: cts } => {
                    let s = match self.index.get(&sender) { Some(&s) => s, None => u32::MAX };
                    if s == u32::MAX {
                        SkgOutcome::PartIgnored  // not a node
                    } else if self.parts.contains_key(&s) {
                        SkgOutcome::PartIgnored  // multiple parts: ignored
                    } else {
                        self.parts.insert(s, Proposal { commit: commit_c48, acks: BTreeSet::new(), values: BTreeMap::new(), our_row: None });
                        match self.our_idx {
                            None => SkgOutcome::PartIgnored,
                            Some(o) if o as usize >= cts.len() || plain.get(&m).map_or(true, |p| p.is_none()) => SkgOutcome::PartIgnored,
                            Some(_) => match (rows.get(&m).cloned().flatten(), row_ok.get(&m).copied().unwrap_or(false)) {
                                (Some(row), true) => {
                                    self.parts.get_mut(&s).unwrap().our_row = Some(row.clone());
                                    SkgOutcome::PartValid { proposer: s, row }
                                }
                                _ => SkgOutcome::PartInvalid(sender),
                            },
                        }
                    }
                }
                SkgMsg::Ack { sender, proposer, values } => {
                    let s = match self.index.get(&sender) { Some(&s) => s, None => u32::MAX };
                    let fault = |kind: &'static str| SkgOutcome::Ack(vec![(sender.clone(), kind)]);
                    if s == u32::MAX {
                        SkgOutcome::Ack(Vec::new())  // not a node
                    } else if values.len() != n {
                        fault("NodeCount")
                    } else if !self.parts.contains_key(&proposer) {
                        fault("SenderExist")
                    } else if self.parts[&proposer].acks.contains(&s) {
                        fault("DuplicateAck")
                    } else {
                        self.parts.get_mut(&proposer).unwrap().acks.insert(s);
                        if self.our_idx.is_none() {
                            SkgOutcome::Ack(Vec::new())
                        } else if plain.get(&m).map_or(true, |p| p.is_none()) {
                            fault("ValueDecryption")
                        } else if vals.get(&m).map_or(true, |v| v.is_none()) {
                            fault("ValueDeserialization")
                        } else if !val_ok.get(&m).copied().unwrap_or(false) {
                            fault("ValueInvalid")
                        } else {
                            let v = vals[&m].unwrap();
                            self.parts.get_mut(&proposer).unwrap().values.insert(s + 1, v);
                            SkgOutcome::Ack(Vec::new())
                        }
                    }
                }
            };
            out.push(outcome);
        }
        Ok(out)
    }
}
