#!/usr/bin/env python3
"""Secondary benchmark lines for the other SURVEY.md §8 configurations (one JSON line each).

bench.py measures the headline metric on C3 (the configuration BASELINE.json's metric is quoted
on).  This script measures the remaining hot-path configurations through the same C ABI, one
GPU, synthetic seeded inputs generated on the device (setup outside the timed region), results
checked against the construction after timing:

  c1  Threshold Coin N=10, f=3 (examples/simulation.rs:43-44, BASELINE config 1), single-call
      latency: one coin's 10 SignatureShares verified, the first t=4 valid ones combined, the
      combined signature checked against the master key and its parity taken (src/coin.rs:
      149-207), from host buffers, each call blocking (the BA epoch waits on its coin,
      binary_agreement.rs:309-323), hash_g2(nonce) on the host inside the call.  Reported beside
      the C restatement of the same call on one core and on every usable core.
  c2  Binary Agreement coins N=100: 100 coin instances x 100 SignatureShares verified
      (PublicKeyShare::verify, src/coin.rs:151) + 100 G2 combines of the first t=34 verified
      shares (combine_signatures + parity, src/coin.rs:185-191,173).  Inputs resident in HBM.
  c4  N=10,000: I coin instances x 10^4 SignatureShares + I G2 Pippenger combines (t=3334).
      BASELINE config 4 shards the I=64 instances over 8 GPUs: `--gpus 8` runs them on a
      one-process node (hbtc_node_*_dev: whole instances per GPU, every GPU verifies and
      combines its own instances, no collective); `--slots 0,0` rehearses the node path with
      two contexts on one GPU.
  c5  SyncKeyGen N=1000, one node's view of an era: 1000 Parts (row.commitment() ==
      commit.row(x), src/sync_key_gen.rs:366), then the 10^6 Acks: each Ack value addressed to
      us decrypted (SecretKey::decrypt = hash_g1_g2 + Ciphertext::verify + sk u + pad,
      :481-484; hbtc_decrypt) and checked (commit.evaluate(x, y) == val*G1, :493).  The SKG
      entry points take host buffers, so this line is PCIe-inclusive (2.7 GB of commitments per
      Part batch); the Parts reuse --distinct bivariate polynomials (laid out per Part in HBM as
      1000 separate copies, so the device work and traffic are those of 1000 Parts), and the
      Ack ciphertexts repeat per distinct (polynomial, sender) value (every Ack is still
      hashed, verified, multiplied and padded on its own).

  bc  Reliable Broadcast of one HoneyBadger epoch at N = 256 (the largest network hbbft's
      reed-solomon-erasure coding accepts: k + p <= 256), one node's view: the N^2 = 65,536 Echo
      proofs it receives validated (Proof::validate, src/broadcast/merkle.rs:82-102, via
      validate_proof, broadcast.rs:255), then the N values decoded (decode_from_shards,
      broadcast.rs:461-493: reconstruct_shards of the f silent nodes' shards, the Merkle tree
      of every instance, the root comparison).  Each proposer's value is --bc-value bytes
      (shard_len = ceil((value + 4) / (N - 2f))).  Inputs resident in HBM; the outputs are
      compared with the proposals after timing.

Usage: python bench_configs.py [--configs c1,c2,c4,c5,bc] [--steps K] [--warmup W]
"""
import argparse
import ctypes
import json
import os
import random
import sys
import time

# 16 HIP hardware queues per process, as bench.py (the library's lanes and streams, plus the node
# path's devices, otherwise share HIP's default 4); HBTC_KEEP_HW_QUEUES=1 keeps the environment's
# value.  Set on import too: the GPU suite runs green with 16 queues for the whole process since
# the per-item exact kernels share one stream.
if not os.environ.get("HBTC_KEEP_HW_QUEUES"):
    os.environ["GPU_MAX_HW_QUEUES"] = "16"

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from hbbft_amd import _native as N  # noqa: E402

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
G1_GEN = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G2_GEN = bytes.fromhex("93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
                       "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")
SEED = 0x6862626674
N_OUT = 6  # output sets rotated per step (bench.py's N_OUT)
STEPS_DEFAULT = {"c1": 50, "c2": 20, "c4": 6, "c5": 1, "bc": 20}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def fr_bytes(vals):
    return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals), dtype=np.uint8).copy()


def key_shares(rng, n):
    """sk_i = poly(i+1) for a random degree-f polynomial (messaging.rs:372-394)."""
    f = (n - 1) // 3
    coeffs = [rng.randrange(1, R) for _ in range(f + 1)]
    sks = []
    for i in range(n):
        acc, x = 0, i + 1
        for c in reversed(coeffs):
            acc = (acc * x + c) % R
        sks.append(acc)
    return coeffs[0], sks


def timed_steps(ctx, fn, steps, warmup):
    ctx.timing_enable(True)
    for _ in range(warmup):
        fn()
    ctx.sync()
    ctx.timing_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    ctx.sync()
    return time.perf_counter() - t0


def breakdown(ctx, steps, fams):
    out = {}
    for f in fams:
        ms, n = ctx.timing_read(f)
        if n:
            out[f] = round(ms / steps, 3)
    return out


MAD_U64_PEAK = 39.32e12  # v_mad_u64_u32 peak at the spec clock (bench.py MAD_U64_PEAK, profiles/r06/intmul_peak.txt)


def roofline_line(ctx, family, kernel, fqm_per_launch, note):
    """The dominant kernel's VALU-integer roofline point: algorithmic Fqm per launch (tools/
    fqm_count.cpp -> bench/roofline_constants.json) x 288 v_mad_u64_u32 / its average HIP-event
    span on its stream (this run)."""
    ms, n = ctx.timing_read(family)
    if not n:
        return None
    avg_s = ms / n / 1e3
    consts = json.load(open(os.path.join(ROOT, "bench", "roofline_constants.json")))
    achieved = fqm_per_launch * consts["mad_u64_u32_per_fqm"] / avg_s / 1e12
    return {"bound": "valu-int (v_mad_u64_u32)", "kernel": kernel, "achieved": round(achieved, 3),
            "peak": MAD_U64_PEAK / 1e12, "unit": "T mad_u64_u32/s",
            "frac": round(achieved / (MAD_U64_PEAK / 1e12), 4), "traffic": None,
            "fqm_per_launch": fqm_per_launch, "kernel_ms_per_launch": round(avg_s * 1e3, 3),
            "kernel_ms_per_launch_source": "HIP-event span on the kernel's stream, this run",
            "work_unit": note}


COIN_FAMS = ["prepare", "sig_verify", "sig_items", "sig_lines", "chk_tiles", "chk_subs",
             "chk_leaves", "rlc_finalize", "lagrange", "comb_decode", "comb_digits", "combine"]


def corrupt_positions(rng, n, n_inst, frac, mode):
    """Wrong shares: `uniform` = a fraction of all shares at random; `senders` = the f Byzantine
    senders (f = (n-1)/3, a random set) sign wrongly in every instance (~33%: BFT's worst case)."""
    total = n * n_inst
    if mode == "senders":
        liars = set(rng.sample(range(n), (n - 1) // 3))
        return [k * n + i for k in range(n_inst) for i in range(n) if i in liars]
    return rng.sample(range(total), int(total * frac))


def coin_inputs(ctx, n, n_inst, corrupt=0.01, corrupt_mode="uniform"):
    """A coin epoch generated on the device (setup): key set, H per instance, shares, expected
    statuses, the master key and the instances' H scalars (for the combine's construction)."""
    rng = random.Random(SEED + n)
    master, sks = key_shares(rng, n)
    pk, st = ctx.g1_mul(G1_GEN, fr_bytes(sks))
    assert not st.any()
    hs = [rng.randrange(1, R) for _ in range(n_inst)]
    H, _ = ctx.g2_mul(G2_GEN, fr_bytes(hs))
    total = n * n_inst
    scal = [sks[i] * h % R for h in hs for i in range(n)]
    expected = np.zeros(total, np.int32)
    for j in corrupt_positions(rng, n, n_inst, corrupt, corrupt_mode):
        scal[j] = (scal[j] + 1) % R
        expected[j] = N.REJECT
    sigs, st = ctx.g2_mul(G2_GEN, fr_bytes(scal))
    assert not st.any()
    return {"pk": pk, "H": H, "sigs": sigs, "expected": expected, "master": master, "hs": hs,
            "offsets": np.arange(0, total + 1, n, dtype=np.uint32),
            "idx": np.tile(np.arange(n, dtype=np.uint32), n_inst), "t": (n - 1) // 3 + 1}


class CoinRunner:
    """The coin epoch on ONE context: every instance's shares verified, then the combines of the
    first t verified shares (hbtc_verify_sig_shares_dev + hbtc_combine_sigs_verified_dev)."""

    def __init__(self, ctx, inp, n_inst):
        self.ctx, self.n_inst, self.t = ctx, n_inst, inp["t"]
        self.offsets = inp["offsets"]
        self.total = int(self.offsets[-1])
        self.ks, bad = ctx.keyset_load(inp["pk"])
        assert bad == 0
        self.d = {}
        for k in ("H", "idx", "sigs"):
            arr = inp[k]
            self.d[k] = ctx.dev_alloc(arr.nbytes)
            ctx.dev_upload(self.d[k], arr)
        # N_OUT output sets rotated per step, as bench.py: the library keeps up to four calls in
        # flight (its lanes, each verification followed by its combine), so step k writes the set
        # whose combine (step k - N_OUT) has long finished
        for j in range(N_OUT):
            self.d["status%d" % j] = ctx.dev_alloc(4 * self.total)
            self.d["out%d" % j] = ctx.dev_alloc(96 * n_inst)
            self.d["par%d" % j] = ctx.dev_alloc(n_inst)
            self.d["cst%d" % j] = ctx.dev_alloc(4 * n_inst)
        self.cur = 0

    def step(self):
        ctx, d, lib, h = self.ctx, self.d, self.ctx.lib, self.ctx.h
        self.cur = (self.cur + 1) % N_OUT
        j = self.cur
        off = N._ptr(self.offsets)
        ctx._check(lib.hbtc_verify_sig_shares_dev(h, self.ks, self.n_inst, d["H"], off, d["idx"], d["sigs"],
                                                  d["status%d" % j]), "verify_sig_shares_dev")
        ctx._check(lib.hbtc_combine_sigs_verified_dev(h, self.n_inst, off, d["idx"], d["sigs"],
                                                      d["status%d" % j], self.t, d["out%d" % j],
                                                      d["par%d" % j], d["cst%d" % j]),
                   "combine_sigs_verified_dev")

    def sync(self):
        self.ctx.sync()

    def results(self):
        j, d, ctx = self.cur, self.d, self.ctx
        st = np.empty(self.total, np.int32)
        out = np.empty(96 * self.n_inst, np.uint8)
        par = np.empty(self.n_inst, np.uint8)
        cst = np.empty(self.n_inst, np.int32)
        for arr, name in ((st, "status"), (out, "out"), (par, "par"), (cst, "cst")):
            ctx.dev_download(arr, d["%s%d" % (name, j)])
        return st, out, par, cst

    def free(self):
        for p in self.d.values():
            self.ctx.dev_free(p)
        self.ctx.keyset_free(self.ks)


class NodeCoinRunner:
    """The same coin epoch on a multi-device node in ONE process (hbtc_node_*): device slot d
    holds whole instances [first[d], first[d+1]) (hbtc_shard_instances, balanced by share
    count) resident in its HBM; each step enqueues every slot's verification and then every
    slot's combine of its own instances (hbtc_node_verify_sig_shares_dev /
    hbtc_node_combine_sigs_verified_dev: one host thread per device for the enqueue, no
    synchronisation).  Instances never cross devices, so there is no exchange: each device's
    verdicts and combined signatures are final where they are computed."""

    def __init__(self, node, inp, n_inst):
        from hbbft_amd import shard
        self.node, self.n_inst, self.t = node, n_inst, inp["t"]
        n_dev = len(node.devices)
        if n_inst < n_dev:
            raise SystemExit("node coin bench: %d instances cannot be split over %d devices as whole "
                             "instances" % (n_inst, n_dev))
        off = inp["offsets"]
        self.total = int(off[-1])
        self.first = [int(x) for x in shard.instance_plan(n_dev, off)]
        self.ks, bad = node.keyset_load(inp["pk"])
        assert bad == 0
        self.ctxs = [node.context(d) for d in range(n_dev)]
        self.slots = []
        for d, c in enumerate(self.ctxs):
            a, b = self.first[d], self.first[d + 1]
            lo, hi = int(off[a]), int(off[b])
            sl = {"a": a, "b": b, "lo": lo, "hi": hi, "offsets": (off[a:b + 1] - off[a]).astype(np.uint32),
                  "mem": {}}
            for name, arr in (("H", inp["H"].reshape(-1, 96)[a:b]), ("idx", inp["idx"][lo:hi]),
                              ("sigs", inp["sigs"].reshape(-1, 96)[lo:hi])):
                arr = np.ascontiguousarray(arr).reshape(-1)
                p = c.dev_alloc(max(arr.nbytes, 16))
                if arr.nbytes:
                    c.dev_upload(p, arr)
                sl["mem"][name] = p
            for j in range(N_OUT):
                for name, nb in (("status", 4 * (hi - lo)), ("out", 96 * (b - a)), ("par", b - a),
                                 ("cst", 4 * (b - a))):
                    sl["mem"]["%s%d" % (name, j)] = c.dev_alloc(max(nb, 16))
            self.slots.append(sl)
        self.parts = []
        for j in range(N_OUT):
            specs = []
            for sl in self.slots:
                m = sl["mem"]
                specs.append({"offsets": sl["offsets"], "d_H_c96": m["H"], "d_idx": m["idx"],
                              "d_items": m["sigs"], "d_status": m["status%d" % j], "d_out": m["out%d" % j],
                              "d_out_parity": m["par%d" % j], "d_inst_status": m["cst%d" % j]})
            self.parts.append(node.parts(specs))
        self.cur = 0

    def step(self):
        self.cur = (self.cur + 1) % N_OUT
        parts, _ = self.parts[self.cur]
        self.node.verify_sig_shares_dev(self.ks, parts)
        self.node.combine_sigs_verified_dev(parts, self.t)

    def sync(self):
        self.node.sync()

    def results(self):
        j = self.cur
        st = np.empty(self.total, np.int32)
        out = np.empty(96 * self.n_inst, np.uint8)
        par = np.empty(self.n_inst, np.uint8)
        cst = np.empty(self.n_inst, np.int32)
        for c, sl in zip(self.ctxs, self.slots):
            a, b, lo, hi, m = sl["a"], sl["b"], sl["lo"], sl["hi"], sl["mem"]
            if b == a:
                continue
            for arr, name, x, y, w in ((st, "status", lo, hi, 1), (out, "out", 96 * a, 96 * b, 1),
                                       (par, "par", a, b, 1), (cst, "cst", a, b, 1)):
                tmp = np.empty(y - x, arr.dtype)
                c.dev_download(tmp, m["%s%d" % (name, j)])
                arr[x:y] = tmp
        return st, out, par, cst

    def free(self):
        for c, sl in zip(self.ctxs, self.slots):
            for p in sl["mem"].values():
                c.dev_free(p)
        self.node.keyset_free(self.ks)


def bench_coins(ctx, name, n, n_inst, steps, warmup, corrupt=0.01, corrupt_mode="uniform", node=None,
                keep_arrays=False, cpu_budget=0.0, latency_steps=0):
    """c2 / c4: n_inst coin instances x n SignatureShares + n_inst combines (first t verified).
    node: a hbtc Node (one process, several device slots) instead of the single context."""
    t0 = time.time()
    inp = coin_inputs(ctx, n, n_inst, corrupt, corrupt_mode)
    t, total = inp["t"], n * n_inst
    run = NodeCoinRunner(node, inp, n_inst) if node is not None else CoinRunner(ctx, inp, n_inst)
    log("%s: setup %.1fs (%d shares%s)" % (name, time.time() - t0, total,
                                           ", node of %d slots" % len(node.devices) if node else ""))
    tctx = run.ctxs[0] if node is not None else ctx
    tctx.timing_enable(True)
    for _ in range(warmup):
        run.step()
    run.sync()
    tctx.timing_reset()
    t1 = time.perf_counter()
    for _ in range(steps):
        run.step()
    run.sync()
    elapsed = time.perf_counter() - t1
    per = breakdown(tctx, steps, COIN_FAMS)
    leaves = tctx.rlc_last_leaves() if ctx_mode[0] == N.MODE_RLC else None
    consts = json.load(open(os.path.join(ROOT, "bench", "roofline_constants.json")))
    items0 = (run.slots[0]["hi"] - run.slots[0]["lo"]) if node is not None else total
    bits = tctx.rlc_bits()
    key = "sig_rlc_item" if bits == 64 or "sig_rlc_item_128" not in consts else "sig_rlc_item_128"
    # (round 6: k_sig_decode_pair + k_sig_items_pair, the G2 arithmetic on lane pairs)
    roof = roofline_line(tctx, "sig_items", "k_sig_decode_pair + k_sig_items_pair", consts[key] * items0,
                         "%s Fqm (G2 decode + subgroup test, [a]s + [b](-psi^2 s), r pk from "
                         "the fixed-base table, tile-tree share) x %d SignatureShares per launch" % (key, items0))
    if roof and node is None:
        # the same step once more with nothing else in flight: the item pass on an idle chip,
        # beside its pipelined span above (where the other lanes' checks and combines share the CUs)
        tctx.timing_reset()
        run.step()
        run.sync()
        iso = roofline_line(tctx, "sig_items", roof["kernel"], roof["fqm_per_launch"], roof["work_unit"])
        if iso:
            roof["kernel_ms_per_launch_isolated"] = iso["kernel_ms_per_launch"]
            roof["frac_isolated"] = iso["frac"]
            roof["isolated_note"] = "one extra step after the timed region with no other step in flight"
    stv, out, par, cst = run.results()
    lat = None
    if node is None and latency_steps:
        # single-call latency: one call at a time (verification + combine, then a sync): what a BA
        # epoch waiting on its coins feels (binary_agreement.rs:309-323, coin.rs:149-181)
        lats = []
        for _ in range(latency_steps):
            a = time.perf_counter()
            run.step()
            run.sync()
            lats.append(time.perf_counter() - a)
        lat = {"p10": round(_pct(lats, 0.1) * 1e3, 3), "median": round(_pct(lats, 0.5) * 1e3, 3),
               "p90": round(_pct(lats, 0.9) * 1e3, 3), "calls": latency_steps,
               "unit": "ms per call (verification + combines, blocking; inputs resident in HBM)"}
        stv, out, par, cst = run.results()
    want, _ = ctx.g2_mul(G2_GEN, fr_bytes([inp["master"] * hh % R for hh in inp["hs"]]))
    mism = int((stv != inp["expected"]).sum())
    comb_ok = bool((cst == 0).all() and bytes(out) == bytes(want))
    if mism or not comb_ok:
        raise SystemExit("%s: results differ from the construction (%d mismatches, combine %s)"
                         % (name, mism, comb_ok))
    run.free()
    n_gpus = len(set(node.devices)) if node is not None else 1
    if node is not None:
        par_s = ("node: one process, %d device slot(s) on %d GPU(s) (hbtc_node_*_dev), whole instances per "
                 "slot (hbtc_shard_instances), each slot verifies and combines its own instances; no "
                 "collective (disjoint outputs)" % (len(node.devices), n_gpus))
    else:
        par_s = "1 GPU"
    res = {
        "metric": "verified BLS12-381 SignatureShares/sec; combines/sec",
        "value": round(total * steps / elapsed, 1), "unit": "shares/s", "n_gpus": n_gpus,
        "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "dtype": "u32 (381-bit Montgomery limbs)",
        "data": "synthetic (seeded key set, shares generated on device; %s)"
                % ("%g%% wrong shares" % (100 * corrupt) if corrupt_mode == "uniform"
                   else "f = %d Byzantine senders sign wrongly in every instance" % ((n - 1) // 3)),
        "mode": "rlc" if ctx_mode[0] == N.MODE_RLC else "per_share",
        "config": {"workload": "%s: %d coin instances x %d SignatureShares verified + %d G2 combines (t=%d)"
                   % (name, n_inst, n, n_inst, t), "N": n, "t": t, "instances": n_inst,
                   "parallelism": par_s},
        "combines_per_s": round(n_inst * steps / elapsed, 2),
        "kernel_event_spans_ms_per_step": per, "mismatches": mism, "combine_ok": comb_ok,
        "exact_single_share_checks_last_call": leaves,
    }
    res["roofline"] = roof
    if lat:
        res["single_call_latency"] = lat
    if node is not None:
        res["kernel_event_spans_note"] = "event spans of device slot 0 only"
    if cpu_budget and node is None:
        try:
            from oracle.cbaseline import run_sig_share_baseline
            nonce = ("Nonce for Honey Badger %s@0:2:0" % ("[" + ", ".join(["0x" + "ab" * 48] * 4) + "]")).encode()
            res["cpu_baseline"] = run_sig_share_baseline(inp["sigs"][:96 * n], inp["pk"], nonce, cpu_budget)
            res["cpu_baseline"]["sample"] += (" (a synthetic %d-byte nonce: hash_g2 of it is not the bench's H, "
                                              "so the pairings reject; the work per share is the same)" % len(nonce))
            if lat:
                from oracle.cbaseline import run_sig_share_baseline as rsb
                one = rsb(inp["sigs"][:96 * n], inp["pk"], nonce, cpu_budget / 2, cores=1)
                res["cpu_baseline"]["single_call_latency_ms"] = {
                    "all_cores": round(1e3 * total / res["cpu_baseline"]["value"], 1),
                    "one_core": round(1e3 * total / one["value"], 1),
                    "note": "projected: the call's %d share checks at the measured per-share rates (the "
                            "%d combines excluded: a lower bound on the reference's call)" % (total, n_inst)}
        except Exception as e:  # the baseline is reported, never the product path
            res["cpu_baseline"] = {"error": repr(e)}
    if keep_arrays:
        res["_arrays"] = (stv, out, par, cst)
    return res


def _pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, int(q * len(s)))]


C1_SKIP = set(filter(None, os.environ.get("HBTC_C1_SKIP", "").split(",")))
COIN_NONCE = (b"Nonce for Honey Badger [173, 84, 2, 11, 0, 0, 9, 254, 1, 18, 200, 57, 43, 9, "
              b"4, 77, 190, 91, 12, 0, 1, 2, 3]@3:2:7")


def bench_c1(ctx, steps, warmup, cpu_budget=0.0):
    """c1: single-call latency of one Threshold Coin at N = 10 (see the docstring)."""
    n, t = 10, 4
    rng = random.Random(SEED + 10)
    master, sks = key_shares(rng, n)
    pk, st = ctx.g1_mul(G1_GEN, fr_bytes(sks))
    mpk, _ = ctx.g1_mul(G1_GEN, fr_bytes([master]))
    H = N.hash_g2(COIN_NONCE)
    scal = list(sks)
    scal[2] = (scal[2] + 1) % R  # one faulty node's wrong share
    sigs, st2 = ctx.g2_mul(H, fr_bytes(scal))
    assert not st.any() and not st2.any()
    expected = np.zeros(n, np.int32)
    expected[2] = N.REJECT
    want_sig, _ = ctx.g2_mul(H, fr_bytes([master]))
    ks, bad = ctx.keyset_load(pk)
    assert bad == 0
    ctx.keyset_set_master(ks, bytes(mpk))
    idx = np.arange(n, dtype=np.uint32)
    sig_list = [bytes(sigs[96 * i:96 * i + 96]) for i in range(n)]

    def call():
        """The coin round as ONE call (hbtc_coin_decide): hash_g2 on the host, then the share
        checks, the combine of the first t verified shares, the master check and the parity."""
        a = time.perf_counter()
        Hc = N.hash_g2(COIN_NONCE)  # host, once per coin instance (north star)
        b = time.perf_counter()
        stv, out, par, cst = ctx.coin_decide(ks, [Hc], [n], idx, sig_list, t)
        e = time.perf_counter()
        return (b - a, e - b, e - a), stv, out[0], int(par[0]), int(cst[0])

    def call_separate():
        """The same coin through the three per-call entry points (verify, combine, PublicKey::verify)."""
        a = time.perf_counter()
        Hc = N.hash_g2(COIN_NONCE)
        b = time.perf_counter()
        stv = ctx.verify_sig_shares(ks, [Hc], [n], idx, sig_list)
        c = time.perf_counter()
        sel = [i for i in range(n) if stv[i] == N.ACCEPT][:t]
        out, par, cst = ctx.combine_sigs([t], sel, [sig_list[i] for i in sel], t)
        d = time.perf_counter()
        ok = ctx.verify_sigs([bytes(mpk)], [Hc], [out[0]])
        e = time.perf_counter()
        return (b - a, c - b, d - c, e - d, e - a), stv, out[0], int(par[0]), int(cst[0]), int(ok[0])

    def call_prepared():
        """hbbft knows the nonce when it creates the Coin (binary_agreement.rs:320), before the
        shares: hash_g2 and H's line tables (hbtc_prepare_g2) then, the coin round on the shares'
        arrival.  Unprepared after every round (each coin has a fresh nonce in hbbft)."""
        a = time.perf_counter()
        Hc = N.hash_g2(COIN_NONCE)
        st_p = ctx.prepare_g2([Hc])
        b = time.perf_counter()
        stv, out, par, cst = ctx.coin_decide(ks, [Hc], [n], idx, sig_list, t)
        e = time.perf_counter()
        ctx.unprepare_g2([Hc])
        assert int(st_p[0]) == N.ACCEPT
        return (b - a, e - b), stv, out[0], int(par[0]), int(cst[0])

    phases = {"hash_g2": [], "coin_decide": []}
    total = []
    for _ in range(warmup):
        call()
    for _ in range(steps):
        ph, stv, sig, par, cst = call()
        phases["hash_g2"].append(ph[0])
        phases["coin_decide"].append(ph[1])
        total.append(ph[2])
    if (stv != expected).any() or cst != N.ACCEPT or sig != bytes(want_sig):
        raise SystemExit("c1: results differ from the construction")
    prep_phases = {"hash_g2_and_prepare": [], "coin_decide": []}
    for _ in range(min(warmup, 2)):
        call_prepared()
    for _ in range(steps):
        ph, stp, sigp, parp, cstp = call_prepared()
        prep_phases["hash_g2_and_prepare"].append(ph[0])
        prep_phases["coin_decide"].append(ph[1])
    if (stp != expected).any() or cstp != N.ACCEPT or sigp != bytes(want_sig) or parp != par:
        raise SystemExit("c1: the prepared round differs from the construction")
    sep_phases = {"hash_g2": [], "verify_shares": [], "combine": [], "verify_master": []}
    sep_total = []
    for _ in range(min(warmup, 2)):
        call_separate()
    for _ in range(max(steps // 2, 5)):
        ph, stv2, sig2, par2, cst2, ok2 = call_separate()
        for k, v in zip(sep_phases, ph[:4]):
            sep_phases[k].append(v)
        sep_total.append(ph[4])
    if (stv2 != expected).any() or cst2 != 0 or ok2 != N.ACCEPT or sig2 != bytes(want_sig) or par2 != par:
        raise SystemExit("c1: the separate calls differ from the construction")
    ctx.keyset_free(ks)
    med = _pct(total, 0.5)
    res = {
        "metric": "Threshold Coin single-call latency at N=10 (verify 10 SignatureShares + combine 4 + "
                  "master verify + parity)",
        "value": round(med * 1e3, 3), "unit": "ms per coin call (median)", "n_gpus": 1, "steps": steps,
        "warmup": warmup, "higher_is_better": False, "dtype": "u32 (381-bit Montgomery limbs)",
        "data": "synthetic (seeded key set, master key; shares sk_i * hash_g2(nonce) made on the device; "
                "node 2's share is wrong)",
        "config": {"workload": "c1: Threshold Coin N=10 f=3 (examples/simulation.rs:43-44): one coin call "
                               "(hbtc_coin_decide), host buffers, blocking", "N": n, "f": 3, "t": t},
        "latency_ms": {"p10": round(_pct(total, 0.1) * 1e3, 3), "median": round(med * 1e3, 3),
                       "p90": round(_pct(total, 0.9) * 1e3, 3)},
        "phase_median_ms": {k: round(_pct(v, 0.5) * 1e3, 3) for k, v in phases.items()},
        "prepared": {"phase_median_ms": {k: round(_pct(v, 0.5) * 1e3, 3) for k, v in prep_phases.items()},
                     "coin_decide_p10_p90_ms": [round(_pct(prep_phases["coin_decide"], 0.1) * 1e3, 3),
                                                round(_pct(prep_phases["coin_decide"], 0.9) * 1e3, 3)],
                     "note": "hash_g2 + hbtc_prepare_g2 when the Coin is created (the nonce is known then, "
                             "binary_agreement.rs:320), timed apart; coin_decide on the shares' arrival with "
                             "H's line tables resident; outputs equal the unprepared round's"},
        "separate_calls": {"median_ms": round(_pct(sep_total, 0.5) * 1e3, 3),
                           "phase_median_ms": {k: round(_pct(v, 0.5) * 1e3, 3) for k, v in sep_phases.items()},
                           "note": "hbtc_verify_sig_shares + hbtc_combine_sigs + hbtc_verify_sigs, each blocking"},
        "calls_per_s": round(1.0 / med, 1),
        "mode": "rlc" if ctx_mode[0] == N.MODE_RLC else "per_share", "results_ok": True,
    }
    if cpu_budget:
        try:
            from oracle.cbaseline import run_coin_call_baseline
            cpu = run_coin_call_baseline(bytes(sigs), bytes(pk), bytes(mpk), COIN_NONCE, t, cpu_budget)
            ok_c, sig_c, par_c = cpu.pop("results")
            cpu["results_equal_gpu"] = bool([not x for x in ok_c] == list(expected == N.REJECT)
                                            and sig_c == bytes(want_sig) and par_c == par)
            res["cpu_baseline"] = cpu
            res["gpu_vs_cpu_latency"] = {
                "gpu_ms": res["value"], "cpu_1core_ms": cpu["value"], "cpu_all_cores_ms": cpu["value_all_cores_ms"],
                "note": "a single N = 10 coin is a chain of a few dependent kernel launches (decode, sums, "
                        "one check level, combine, master check) on an idle GPU; the CPU does 11 pairing checks"}
        except Exception as e:  # reported, never the product path
            res["cpu_baseline"] = {"error": repr(e)}
    return res


def bench_skg(ctx, n, n_parts, n_distinct, steps, warmup, cpu_budget=0.0):
    """c5: one node's SyncKeyGen view at N=n (t = (n-1)/3): n_parts Parts, then n_parts x n Acks."""
    rng = random.Random(SEED + 5)
    t0 = time.time()
    t = (n - 1) // 3
    t1, m = t + 1, (t + 1) * (t + 2) // 2
    our = 17
    x = our + 1
    polys = [[rng.randrange(R) for _ in range(m)] for _ in range(n_distinct)]
    commit_d = []
    for b in polys:
        c, st = ctx.g1_mul(G1_GEN, fr_bytes(b))
        assert not st.any()
        commit_d.append(c)
    xp = [pow(x, j, R) for j in range(t1)]

    def pos(i, j):
        return j * (j + 1) // 2 + i if j >= i else i * (i + 1) // 2 + j

    rows_d = [[sum(b[pos(i, j)] * xp[j] for j in range(t1)) % R for i in range(t1)] for b in polys]

    def horner(row, y):
        acc = 0
        for c in reversed(row):
            acc = (acc * y + c) % R
        return acc

    vals_d = [[horner(r, s + 1) for s in range(n)] for r in rows_d]
    commits = np.concatenate([commit_d[p % n_distinct] for p in range(n_parts)])
    rows = [list(rows_d[p % n_distinct]) for p in range(n_parts)]
    bad_part = 7 % n_parts
    rows[bad_part][t // 2] = (rows[bad_part][t // 2] + 1) % R
    rows_b = fr_bytes([v for r in rows for v in r])
    part_expect = np.full(n_parts, N.ACCEPT, np.int32)
    part_expect[bad_part] = N.REJECT
    n_acks = n_parts * n
    ack_part = np.repeat(np.arange(n_parts, dtype=np.uint32), n)
    ack_sender = np.tile(np.arange(n, dtype=np.uint32), n_parts)
    vals_d_b = [fr_bytes(v).reshape(n, 32) for v in vals_d]
    vals = np.concatenate([vals_d_b[p % n_distinct] for p in range(n_parts)]).reshape(n_acks, 32)
    ack_expect = np.full(n_acks, N.ACCEPT, np.int32)
    for a in rng.sample(range(n_acks), 100):  # tampered values (ValueInvalid)
        v = (int.from_bytes(vals[a].tobytes(), "little") + 1) % R
        vals[a] = np.frombuffer(v.to_bytes(32, "little"), np.uint8)
        ack_expect[a] = N.REJECT
    vals = vals.reshape(-1)
    # the Ack values addressed to us, encrypted to our key (one ciphertext per distinct value)
    from hbbft_amd import skg, wire
    our_sk = rng.randrange(1, R)
    our_pk, _ = ctx.g1_mul(G1_GEN, fr_bytes([our_sk]))
    vmat = vals.reshape(n_acks, 32)
    keyof = {}
    for a in range(n_acks):
        keyof.setdefault(vmat[a].tobytes(), len(keyof))
    distinct = [None] * len(keyof)
    for k, j in keyof.items():
        distinct[j] = wire.fr_to_wire(int.from_bytes(k, "little"))
    pool = skg.encrypt_batch(ctx, [bytes(our_pk)] * len(distinct), distinct)
    which = np.array([keyof[vmat[a].tobytes()] for a in range(n_acks)], np.int64)
    pu = np.frombuffer(b"".join(c.u for c in pool), np.uint8).reshape(-1, 48)
    pw = np.frombuffer(b"".join(c.w for c in pool), np.uint8).reshape(-1, 96)
    pv = np.frombuffer(b"".join(c.v for c in pool), np.uint8).reshape(-1, 40)
    ack_u, ack_w, ack_v = (np.ascontiguousarray(x[which]).reshape(-1) for x in (pu, pw, pv))
    ack_off = np.arange(0, 40 * n_acks + 1, 40, dtype=np.uint32)
    ack_plain = np.empty(40 * n_acks, np.uint8)
    ack_dst = np.empty(n_acks, np.int32)
    sk_b = fr_bytes([our_sk])
    log("c5: setup %.1fs (%d Parts x %d commitment points, %d Acks, %d distinct Ack ciphertexts)"
        % (time.time() - t0, n_parts, m, n_acks, len(pool)))
    lib, h = ctx.lib, ctx.h
    pst = np.empty(n_parts, np.int32)
    ast = np.empty(n_acks, np.int32)
    row_ok = np.empty(n_parts, np.uint8)
    t_parts = [0.0]
    t_dec = [0.0]
    dec_vals = np.empty(32 * n_acks, np.uint8)

    def step():
        a0 = time.perf_counter()
        ctx._check(lib.hbtc_skg_check_parts(h, n_parts, t, our, N._ptr(commits), N._ptr(rows_b),
                                            N._ptr(pst)), "skg_check_parts")
        a1 = time.perf_counter()
        t_parts[0] += a1 - a0
        row_ok[:] = (pst == N.ACCEPT)
        # our value of every Ack: SecretKey::decrypt, then the FieldWrap<Fr> framing (32-byte BE)
        ctx._check(lib.hbtc_decrypt(h, n_acks, N._ptr(sk_b), N._ptr(ack_u), N._ptr(ack_w),
                                    N._ptr(ack_v), N._ptr(ack_off), N._ptr(ack_plain),
                                    N._ptr(ack_dst)), "decrypt")
        dec_vals.reshape(n_acks, 32)[:] = ack_plain.reshape(n_acks, 40)[:, 8:][:, ::-1]
        t_dec[0] += time.perf_counter() - a1
        ctx._check(lib.hbtc_skg_check_acks(h, n_parts, t, our, N._ptr(commits), N._ptr(rows_b),
                                           N._ptr(row_ok), n_acks, N._ptr(ack_part),
                                           N._ptr(ack_sender), N._ptr(dec_vals), N._ptr(ast)),
                   "skg_check_acks")

    for _ in range(warmup):
        step()
    t_parts[0] = t_dec[0] = 0.0
    elapsed = timed_steps(ctx, step, steps, 0)
    per = breakdown(ctx, steps, ["skg_scalars", "skg_ack_rows", "comb_decode", "comb_digits",
                                 "combine", "mul", "hash", "pb_items", "pb_lines", "pb_ml", "pb_checks", "pair_verify"])
    pm = int((pst != part_expect).sum())
    am = int((ast != ack_expect).sum()) + int((ack_dst != N.ACCEPT).sum())
    if pm or am:
        raise SystemExit("c5: results differ from the construction (%d Part, %d Ack mismatches)" % (pm, am))
    consts = json.load(open(os.path.join(ROOT, "bench", "roofline_constants.json")))
    dec_ms, dec_n = ctx.timing_read("comb_decode")
    # decodes per step: every Part's commitment (n_parts x m points), plus the commitment of each
    # Part whose row failed (its Acks go through an RLC MSM over the commitment again)
    n_dec = (n_parts + int((part_expect != N.ACCEPT).sum())) * m
    roof = roofline_line(ctx, "comb_decode", "k_msm_decode<Fq, 12>",
                         consts["dec_share"]["decode"] * n_dec * steps // max(dec_n, 1),
                         "G1 decode + subgroup test Fqm (dec_share.decode) x the commitment points one "
                         "launch decodes (%d per step over %d launches)" % (n_dec, dec_n // max(steps, 1)))
    cpu = None
    if cpu_budget:
        try:
            from oracle.cbaseline import run_skg_ack_baseline
            cpu = run_skg_ack_baseline(n, t, cpu_budget)
        except Exception as e:  # reported, never the product path
            cpu = {"error": repr(e)}
    tp = t_parts[0] / steps
    td = t_dec[0] / steps
    ta = elapsed / steps - tp
    return {
        "metric": "SyncKeyGen checks/sec: Parts/s and Acks/s (one node's view)",
        "value": round(n_acks * steps / elapsed, 1), "unit": "acks/s (Parts + Acks of the era in the timed region)",
        "n_gpus": 1, "steps": steps, "warmup": warmup, "ms_per_step": round(elapsed / steps * 1e3, 3),
        "higher_is_better": True, "dtype": "u32 (381-bit Montgomery limbs)",
        "data": "synthetic (%d distinct bivariate polynomials reused over %d Parts; 1 Part with a tampered row, 100 tampered Ack values; %d distinct Ack ciphertexts); host buffers (PCIe-inclusive)"
                % (n_distinct, n_parts, len(pool)),
        "config": {"workload": "c5: SyncKeyGen N=%d: %d Parts (%d-point BivarCommitments) + %d Acks (decrypt + value check)"
                   % (n, n_parts, m, n_acks), "N": n, "t": t, "parts": n_parts, "acks": n_acks},
        "parts_ms": round(tp * 1e3, 3), "acks_ms": round(ta * 1e3, 3),
        "acks_decrypt_ms": round(td * 1e3, 3),
        "parts_per_s": round(n_parts / tp, 1), "acks_per_s": round(n_acks / ta, 1),
        "kernel_event_spans_ms_per_step": per, "mismatches": pm + am,
        "roofline": roof, "cpu_baseline": cpu,
    }


def bench_broadcast(ctx, n, value_bytes, steps, warmup):
    """bc: one node's Reliable Broadcast work for an epoch of n proposers (see the docstring)."""
    from hbbft_amd import broadcast as G
    lib, h = ctx.lib, ctx.h
    rng = np.random.default_rng(SEED + n)
    f = (n - 1) // 3
    k, p = G.shard_counts(n, f)
    t0 = time.time()
    values = [rng.integers(0, 256, value_bytes, dtype=np.uint8).tobytes() for _ in range(n)]
    shards = G.encode_batch(ctx, values, n, f)               # [n_inst, n, L] (setup)
    L = shards.shape[2]
    nd = lib.hbtc_merkle_digest_count(n)
    dig = ctx.merkle_trees(n, L, shards.reshape(-1))        # [n_inst, nd, 32]
    roots = dig[:, -1, :].copy()
    # the Echo proofs this node receives: node j's proof of instance kk, for every (kk, j)
    lvl_off, m, off = [], n, 0
    while m > 1:
        lvl_off.append((off, m))
        off += m
        m = (m + 1) // 2
    per = []
    for j in range(n):
        pos, i = [], j
        for o, size in lvl_off:
            if (i ^ 1) < size:
                pos.append(o + (i ^ 1))
            i //= 2
        per.append(pos)
    depth = np.array([len(x) for x in per], np.uint32)
    n_pr = n * n
    doff = np.zeros(n_pr + 1, np.uint32)
    doff[1:] = np.cumsum(np.tile(depth, n))
    digs = np.concatenate([dig[kk][per[j]] for kk in range(n) for j in range(n)]).reshape(-1)
    voff = (np.arange(n_pr + 1, dtype=np.uint64) * L).astype(np.uint64)
    idx = np.tile(np.arange(n, dtype=np.uint32), n)
    proot = np.repeat(roots, n, axis=0).reshape(-1)
    # this node's view for decoding: the f silent nodes' shards are missing in every instance
    silent = rng.choice(n, f, replace=False)
    present = np.ones((n, n), np.uint8)
    present[:, silent] = 0
    recv = shards.copy()
    recv[:, silent, :] = 0
    d = {}
    for name, arr in (("values", shards.reshape(-1)), ("voff", voff), ("idx", idx), ("doff", doff),
                      ("digs", digs), ("roots", proot), ("recv", recv.reshape(-1))):
        d[name] = ctx.dev_alloc(arr.nbytes)
        ctx.dev_upload(d[name], arr)
    d["status"] = ctx.dev_alloc(4 * n_pr)
    d["out"] = ctx.dev_alloc(n * nd * 32)
    rstatus = np.empty(n, np.int32)
    log("bc: setup %.1fs (%d proofs, %d instances, shard_len %d)" % (time.time() - t0, n_pr, n, L))

    # HBTC_BC_PHASE_SYNC=1: a sync between the phases, so each kernel's duration in a trace is
    # its own (by default the three calls run on different verification lanes and overlap)
    phase_sync = os.environ.get("HBTC_BC_PHASE_SYNC") == "1"

    def step():
        ctx._check(lib.hbtc_merkle_validate_dev(h, n_pr, n, d["voff"], d["values"], d["idx"], d["doff"],
                                                d["digs"], d["roots"], d["status"]), "validate")
        if phase_sync:
            ctx.sync()
        ctx._check(lib.hbtc_rs_reconstruct_dev(h, k, p, L, n, d["recv"], N._ptr(present.reshape(-1)),
                                               N._ptr(rstatus)), "reconstruct")
        if phase_sync:
            ctx.sync()
        ctx._check(lib.hbtc_merkle_trees_dev(h, n, L, n, d["recv"], d["out"]), "trees")
        if phase_sync:
            ctx.sync()

    dt = timed_steps(ctx, step, steps, warmup)
    per_step = breakdown(ctx, steps, ["merkle_validate", "rs", "merkle"])
    st = np.empty(n_pr, np.int32)
    ctx.dev_download(st, d["status"])
    out = np.empty(n * nd * 32, np.uint8)
    ctx.dev_download(out, d["out"])
    rec = np.empty(recv.size, np.uint8)
    ctx.dev_download(rec, d["recv"])
    ctx.sync()
    ok = bool((st == N.ACCEPT).all()) and bool((rstatus == N.ACCEPT).all())
    ok = ok and bool((out.reshape(n, nd, 32)[:, -1, :] == roots).all())
    rec = rec.reshape(n, n, L)
    ok = ok and all(G.glue_shards([bytes(rec[kk, j]) for j in range(k)], k) == values[kk] for kk in range(n))
    for v in d.values():
        ctx.dev_free(v)
    # CPU baseline: the restatement (oracle/broadcast.py: hashlib SHA3, numpy GF(2^8)) on one
    # core over a bounded sample of the same work: 2048 proofs and 2 decodes
    from oracle import broadcast as B
    t1 = time.perf_counter()
    n_cpu = 2048
    for q in range(n_cpu):
        kk, j = divmod(q, n)
        dg = [bytes(dig[kk][x]) for x in per[j]]
        assert B.proof_validate((bytes(shards[kk, j]), j, dg, bytes(roots[kk])), n)
    t_val = (time.perf_counter() - t1) / n_cpu
    t1 = time.perf_counter()
    for kk in range(2):
        lv = [None if j in set(silent.tolist()) else bytes(shards[kk, j]) for j in range(n)]
        assert B.decode_from_shards(lv, f, bytes(roots[kk])) == values[kk]
    t_dec = (time.perf_counter() - t1) / 2
    cpu_step = t_val * n_pr + t_dec * n
    ms = dt / steps * 1e3
    return {
        "metric": "Reliable Broadcast Echo proofs validated/sec (one node, N=256); values decoded/sec",
        "value": round(n_pr / (dt / steps), 1), "unit": "proofs/s", "n_gpus": 1, "steps": steps,
        "warmup": warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "dtype": "u8 / u64 (GF(2^8), Keccak-f[1600])",
        "data": "synthetic (seeded random proposals, f silent nodes)",
        "config": {"workload": "bc: %d Echo proofs validated + %d values decoded (reconstruct %d missing "
                               "shards of %d, Merkle tree, root check)" % (n_pr, n, f, n),
                   "N": n, "f": f, "data_shards": k, "parity_shards": p, "value_bytes": value_bytes,
                   "shard_len": L},
        "values_decoded_per_s": round(n / (dt / steps), 1),
        "input_bytes_per_step": int(n_pr * L + digs.size + n * (n - f) * L),
        "kernel_event_spans_ms_per_step": per_step, "results_ok": ok,
        "cpu_baseline": {"value": round(n_pr / cpu_step, 1), "unit": "proofs/s (with the epoch's decodes)",
                         "cores": 1, "kind": "port",
                         "sample": "2048 Proof::validate + 2 decode_from_shards (first call builds the "
                                   "decode matrix) by oracle/broadcast.py, scaled to the epoch: "
                                   "%.1f us/proof, %.1f ms/decode" % (t_val * 1e6, t_dec * 1e3)},
    }


ctx_mode = [None]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="c1,c2,c4,c5")
    ap.add_argument("--steps", type=int, default=None,
                    help="timed steps (default per config: c2 20, c4 6, c5 1, bc 20 -- enough "
                         "for the pipelined calls to reach steady state)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed steps (default 2; c5 1)")
    ap.add_argument("--inst", type=int, default=64, help="c4 coin instances (of the whole node)")
    ap.add_argument("--gpus", type=int, default=1,
                    help="c2 / c4: devices of a one-process node (hbtc_node_*_dev, whole instances per "
                         "GPU); 1 = a single context")
    ap.add_argument("--slots", default=None,
                    help="c2 / c4: explicit device slots of the node, e.g. 0,0 (two contexts on GPU 0: "
                         "a rehearsal of the node path on one GPU)")
    ap.add_argument("--parts", type=int, default=1000, help="c5 Parts")
    ap.add_argument("--distinct", type=int, default=4, help="c5 distinct bivariate polynomials")
    ap.add_argument("--bc-value", type=int, default=65536, help="bc: bytes per proposed value")
    ap.add_argument("--mode", choices=["rlc", "per_share"], default="rlc")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baselines")
    ap.add_argument("--corrupt", type=float, default=0.01)
    ap.add_argument("--corrupt-mode", choices=["uniform", "senders"], default="uniform")
    args = ap.parse_args()
    ctx = N.Context(0)
    ctx_mode[0] = N.MODE_RLC if args.mode == "rlc" else N.MODE_PER_SHARE
    ctx.set_verify_mode(ctx_mode[0])
    node = None
    slots = [int(x) for x in args.slots.split(",")] if args.slots else list(range(args.gpus))
    if len(slots) > 1:
        node = N.Node(slots)
        node.set_verify_mode(ctx_mode[0])
    try:
        for c in args.configs.split(","):
            steps = args.steps if args.steps is not None else STEPS_DEFAULT.get(c, 2)
            warmup = args.warmup if args.warmup is not None else (1 if c == "c5" else 2)
            if c == "c1":
                out = bench_c1(ctx, steps, warmup, cpu_budget=0.0 if args.no_cpu else 10.0)
            elif c == "c2":
                out = bench_coins(ctx, "c2", 100, 100, steps, warmup, args.corrupt,
                                  args.corrupt_mode, node=node, cpu_budget=0.0 if args.no_cpu else 10.0,
                                  latency_steps=20)
            elif c == "c4":
                out = bench_coins(ctx, "c4", 10000, args.inst, steps, warmup, args.corrupt,
                                  args.corrupt_mode, node=node, cpu_budget=0.0 if args.no_cpu else 10.0)
            elif c == "bc":
                out = bench_broadcast(ctx, 256, args.bc_value, steps, warmup)
            elif c == "c5":
                out = bench_skg(ctx, 1000, args.parts, args.distinct, steps, warmup,
                                cpu_budget=0.0 if args.no_cpu else 10.0)
            else:
                raise SystemExit("unknown config " + c)
            if out is not None:
                print(json.dumps(out), flush=True)
    finally:
        if node is not None:
            node.close()
        ctx.close()


if __name__ == "__main__":
    main()
