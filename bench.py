#!/usr/bin/env python3
"""Benchmark: verified BLS12-381 shares/sec (whole node) at N=1000 + combines/sec.

Workload (BASELINE.json configs[2], the configuration the metric is quoted on, "at N=1000"):
one HoneyBadger epoch = 1000 ciphertexts x 1000 DecryptionShares (every share of every
ciphertext verified: e(share_i, H_ct) == e(pk_i, w_ct), src/threshold_decryption.rs:159) plus
the 1000 G1 Lagrange combines of the first t = 334 VERIFIED shares of every ciphertext
(PublicKeySet::decrypt, td.rs:184), one batched Pippenger MSM launch sequence.
A step = one such epoch through the HIP path; inputs (compressed shares as on the wire, per-
ciphertext H = hash_g1_g2(u, v) and w, the node index of every share) are already resident in
HBM when the timed region starts; decode + subgroup checks are inside it.  ~1% of shares are
corrupted (valid points, wrong share) and a few carry invalid encodings; decisions are checked
against the construction after timing.

Multi-GPU (strong scaling, the default for --gpus N > 1): one process per GPU
(torch.distributed.run), the SAME C3 epoch split over the ranks by hbtc_shard_instances (whole
ciphertexts, balanced by share count; hbbft_amd/shard.py): every rank verifies and combines its
ciphertexts, then one RCCL all-gather over xGMI merges the verdicts and combined points into the
whole epoch's arrays on every rank (the north star's only collective), ordered behind the
library's streams with hbtc_stream_wait_ctx.  The merged epoch is checked against the
construction after timing.  --scaling weak runs an independent 1000-ciphertext epoch per rank
instead (no collective).

Prints ONE JSON line on rank 0 (contract in the task statement), with "roofline" (the longest
critical-path kernel of the default RLC mode; Fqm counted by tools/fqm_count.cpp ->
bench/roofline_constants.json; HBM traffic from the committed PMC passes), "cpu_baseline" (the
oracle's threshold_crypto restatement timed on this host), and at N = 1 two more measured
lines: "adversarial" (f = 333 Byzantine senders send wrong shares on every ciphertext, BFT's
worst case) and "host_buffers" (the same epoch through the host-buffer entry points: H2D of
the compressed shares and D2H of the verdicts inside the timed region).
"""
import argparse
import ctypes
import json
import os
import random
import sys
import time

# HIP hardware queues per process, read once at the first HIP call: the library's four lanes x
# (verification + preparation) streams plus the strong-scaling merge's torch / RCCL streams
# share HIP's default 4 queues, and a gather stream's wait on every lane then blocks the lane
# work queued behind it on the same queue: the merge at world size 1 cost 28.0 vs 16.5 ms per
# 125-ciphertext slice and 101.7 vs 79.6 ms per C3 epoch; with 16 queues 17.7 / 80.0 ms, plain
# runs unchanged (profiles/r03/hw_queues/).  HBTC_KEEP_HW_QUEUES=1 keeps the environment's value.
# Set on import too (a test process importing this module gets 16 queues for the whole process):
# round 3's suite failed that way because the per-item exact kernels' ~6 KB/lane of scratch was
# reserved on every queue they ran on; they now share one stream, and the suite
# runs green with 16 queues (profiles/r04/run6/).
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
# The VALU integer-multiply roofline of the Fqm kernels: v_mad_u64_u32 issues at 4 cycles per
# wave-instruction per SIMD (16 lane-ops / cycle; tools/microbench/intmul.hip measures 4.15-4.2
# including its loop, at 2 to 8 waves per SIMD), so at the 2.4 GHz spec clock the chip's peak is
# 256 CUs x 4 SIMDs x 16 x 2.4e9 = 39.32 T lane-ops/s.  The harness that measures it reaches 72.1 T
# packed-FMA lane-ops/s = 0.92 of the 78.6 T behind the 157.3 TFLOP/s FP32 spec (its sanity line);
# under an integer-multiply load the chip holds 2.15-2.28 GHz, where the same harness delivers
# 35.6 T v_mad_u64_u32/s.  profiles/r06/intmul_peak.txt.  (Rounds 1-5 divided by the round-1
# harness's 29.51 T, which under-drove the instruction: every earlier frac reads ~1.33x high.)
MAD_U64_PEAK = 39.32e12
MAD_U64_PEAK_NOTE = ("v_mad_u64_u32 at 4 cycles per wave-instruction per SIMD x 1024 SIMDs x 64 lanes x 2.4 GHz "
                     "spec clock; tools/microbench/intmul.hip: 4.15-4.2 cyc/insn measured (35.6 T at the 2.28 GHz "
                     "the chip holds under load), sanity line v_pk_fma_f32 72.1 T lane-FMA/s = 0.92 of the FP32 "
                     "spec; profiles/r06/intmul_peak.txt")
# timing family -> kernel (hbtc_api.hip timed() families, rocprofv3 names), per check schedule
# (hbtc_check_schedule_for: the plain-first form for calls that fill the chip, the paired forms
# for small calls such as a rank's slice of the epoch)
KERNEL_NAME_COMMON = {"dec_verify": "k_dec_verify", "rlc_items": "k_rlc_items", "chk_leaves": "k_chk_leaves"}
KERNEL_NAME_SCHED = {
    0: {"chk_tiles": "k_chk_plain<0>", "chk_tiles_w": "k_chk_weighted<0>", "chk_halves": "k_chk_halves",
        "chk_halves_w": "k_chk_weighted<2>", "chk_subs": "k_chk_plain<3>", "chk_subs_w": "k_chk_weighted<3>"},
    1: {"chk_tiles": "k_chk_pair<0, false>", "chk_subs": "k_chk_pair<1, true>"},
    2: {"chk_tiles": "k_chk_pair<0, true>"},
}
# families launched as more than one kernel (hbtc_rlc.hip HBTC_RLC_SPLIT: k_rlc_decode at three waves
# per SIMD, then the scalar half k_rlc_items)
KERNEL_PARTS = {"rlc_items": ("k_rlc_decode", "k_rlc_items")}
SCHED_NAME = {0: "plain-first", 1: "paired: tiles -> sub-tiles -> leaves", 2: "paired: tiles -> leaves"}


def kernel_names(schedule):
    k = dict(KERNEL_NAME_COMMON)
    k.update(KERNEL_NAME_SCHED[schedule])
    return k


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scalars_bytes(vals):
    return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals), dtype=np.uint8).copy()


class Epoch:
    """Synthetic C3 epoch, generated on the GPU with the library's batched scalar multiplication
    (setup, outside the timed region).  Every ciphertext k's data derives from (seed, k) alone,
    so a rank holding ciphertexts [a, b) of a sharded epoch has exactly the rows the one-GPU
    epoch has there; the key set and the corruption pattern are global.

    corrupt_mode "uniform": round(corrupt * n) wrong shares (valid points, wrong scalar) in every
    ciphertext; "senders": the f Byzantine senders send wrong shares on every ciphertext.  Plus 8
    shares of the whole epoch with an invalid encoding."""

    def __init__(self, ctx, n, n_ct, seed, corrupt_frac=0.01, corrupt_mode="uniform", ct_range=None,
                 out_alloc=None, load_keyset=True):
        rng = random.Random(seed)
        self.n, self.n_ct = n, n_ct
        self.f = (n - 1) // 3
        self.t = self.f + 1
        coeffs = [rng.randrange(1, R) for _ in range(self.f + 1)]
        self.master_sk = coeffs[0]
        sks = []
        for i in range(n):
            acc = 0
            for c in reversed(coeffs):
                acc = (acc * (i + 1) + c) % R
            sks.append(acc)
        liars = set(rng.sample(range(n), self.f)) if corrupt_mode == "senders" else set()
        enc_bad = set(rng.sample(range(n * n_ct), 8))
        a, b = ct_range or (0, n_ct)
        self.a, self.b = a, b
        pk, st = ctx.g1_mul(G1_GEN, scalars_bytes(sks))
        assert not st.any()
        self.pk = pk
        self.keyset = None
        if load_keyset:  # (a node loads the key set on every device itself)
            self.keyset, bad = ctx.keyset_load(pk)
            assert bad == 0
        rs, hs = [], []
        for k in range(a, b):
            rk = random.Random(seed * 1000003 + k)
            rs.append(rk.randrange(1, R))
            hs.append(rk.randrange(1, R))
        self.rs = rs
        H, _ = ctx.g2_mul(G2_GEN, scalars_bytes(hs))
        w, _ = ctx.g2_mul(G2_GEN, scalars_bytes([r * h % R for r, h in zip(rs, hs)]))
        u, _ = ctx.g1_mul(G1_GEN, scalars_bytes(rs))
        self.H, self.w = H, w
        self.pk_bytes = [bytes(pk[48 * i:48 * i + 48]) for i in range(n)]
        self.u_bytes = [bytes(u[48 * k:48 * k + 48]) for k in range(b - a)]
        self.w_bytes = [bytes(w[96 * k:96 * k + 96]) for k in range(b - a)]
        m = b - a
        total = n * m
        scal = [sks[i] * r % R for r in rs for i in range(n)]
        self.expected = np.zeros(total, np.int32)
        n_wrong = int(round(n * corrupt_frac)) if corrupt_mode == "uniform" else 0
        for kk in range(m):
            k = a + kk
            wrong = liars or random.Random(seed * 1000003 + k + 0x5EED).sample(range(n), n_wrong)
            for i in wrong:
                j = kk * n + i
                scal[j] = (scal[j] + 1) % R
                self.expected[j] = N.REJECT
        shares, st = ctx.g1_mul(G1_GEN, scalars_bytes(scal))
        assert not st.any()
        shares = shares.reshape(total, 48)
        for g in enc_bad:
            if a * n <= g < b * n:
                shares[g - a * n, 0] &= 0x7F  # clear the compression flag: pairing 0.14 rejects it
                self.expected[g - a * n] = N.DECODE_ERR
        self.offsets = np.arange(0, total + 1, n, dtype=np.uint32)
        self.idx = np.tile(np.arange(n, dtype=np.uint32), m)
        # resident device copies
        self.d = {}
        for name, arr in (("H", H), ("w", w), ("idx", self.idx), ("shares", shares.reshape(-1))):
            p = ctx.dev_alloc(arr.nbytes)
            ctx.dev_upload(p, arr)
            self.d[name] = p
        # N_OUT sets of outputs, rotated per step: the library keeps up to four epochs in flight
        # (its four lanes, each verification followed by its combine), and under strong scaling
        # the all-gather of a set runs after them, so epoch k writes the set epoch k-N_OUT's
        # combine and gather have long finished with
        alloc = out_alloc or (lambda nbytes, i32: (ctx.dev_alloc(nbytes), None))
        self.out = []
        for j in range(N_OUT):
            self.out.append({name: alloc(nb, i32) for name, nb, i32 in
                             (("status", 4 * total, True), ("g", 48 * m, False), ("cst", 4 * m, True))})
        self.cur = 0
        self.m = m
        self.total = total
        self.host_shares = shares

    def ptr(self, j, name):
        return self.out[j][name][0]

    def step(self, ctx):
        """One epoch: the share checks, then the combines of the first t VERIFIED shares of
        every ciphertext (PublicKeySet::decrypt over ThresholdDecryption's verified share map,
        td.rs:184).  The combines run on the verification's lane behind it, while the next epochs'
        verifications run on the library's other lanes (pipelined epochs)."""
        lib, h, d = ctx.lib, ctx.h, self.d
        self.cur = (self.cur + 1) % N_OUT
        j = self.cur
        off = N._ptr(self.offsets)
        ctx._check(lib.hbtc_verify_dec_shares_dev(h, self.keyset, self.m, d["H"], d["w"], off,
                                                  d["idx"], d["shares"], self.ptr(j, "status")),
                   "verify_dec_shares_dev")
        ctx._check(lib.hbtc_combine_dec_verified_dev(h, self.m, off, d["idx"], d["shares"],
                                                     self.ptr(j, "status"), self.t, self.ptr(j, "g"),
                                                     self.ptr(j, "cst")),
                   "combine_dec_verified_dev")

    def results(self, ctx, j=None):
        """(status, g, cst) of the last step (host arrays)."""
        j = self.cur if j is None else j
        st = np.empty(self.total, np.int32)
        g = np.empty(48 * self.m, np.uint8)
        cst = np.empty(self.m, np.int32)
        for arr, name in ((st, "status"), (g, "g"), (cst, "cst")):
            ctx.dev_download(arr, self.ptr(j, name))
        return st, g, cst

    def want_g(self, ctx):
        want, _ = ctx.g1_mul(G1_GEN, scalars_bytes([self.master_sk * r % R for r in self.rs]))
        return want

    def check(self, ctx):
        st, g, cst = self.results(ctx)
        mism = int((st != self.expected).sum())
        comb_ok = bool((cst == 0).all() and bytes(g) == bytes(self.want_g(ctx)))
        return mism, comb_ok, int((st == N.ACCEPT).sum())

    def free(self, ctx):
        for p in self.d.values():
            ctx.dev_free(p)
        for o in self.out:
            for p, t in o.values():
                if t is None:
                    ctx.dev_free(p)
        if self.keyset is not None:
            ctx.keyset_free(self.keyset)


class StrongGather:
    """The merge of a sharded epoch: after a rank's verification + combines, one all-gather of
    the statuses, combined points and combine statuses (RCCL over xGMI; hbbft_amd/shard.py).
    Gathers of output set j run on torch stream j, ordered after the library's streams
    (hbtc_stream_wait_ctx); the library writes output set j again only after stream j's gather
    has read it (hbtc_ctx_wait_stream)."""

    def __init__(self, ep, dist, slices, torch):
        self.ep, self.dist, self.torch = ep, dist, torch
        self.len_items = [hi - lo for _, (lo, hi) in slices]
        self.len_cts = [b - a for (a, b), _ in slices]
        dev = torch.device("cuda", torch.cuda.current_device())
        self.streams = [torch.cuda.Stream(dev) for _ in range(N_OUT)]
        tot_items, tot_cts = sum(self.len_items), sum(self.len_cts)
        self.all = [{"status": torch.empty(tot_items, dtype=torch.int32, device=dev),
                     "g": torch.empty((tot_cts, 48), dtype=torch.uint8, device=dev),
                     "cst": torch.empty(tot_cts, dtype=torch.int32, device=dev)} for _ in range(N_OUT)]

    def before_step(self, ctx):
        if "wait" not in DIAG_SKIP:
            ctx.ctx_wait_stream(self.streams[(self.ep.cur + 1) % N_OUT].cuda_stream)

    def after_step(self, ctx):
        from hbbft_amd import shard
        j = self.ep.cur
        s = self.streams[j]
        if "order" not in DIAG_SKIP:
            ctx.stream_wait_ctx(s.cuda_stream)
        if "gather" in DIAG_SKIP:
            return
        out = self.ep.out[j]
        with self.torch.cuda.stream(s):
            shard.gather_slices(self.dist, out["status"][1], self.len_items, out=self.all[j]["status"])
            shard.gather_slices(self.dist, out["g"][1].view(-1, 48), self.len_cts, out=self.all[j]["g"])
            shard.gather_slices(self.dist, out["cst"][1], self.len_cts, out=self.all[j]["cst"])

    def merged(self):
        self.torch.cuda.synchronize()
        a = self.all[self.ep.cur]
        return a["status"].cpu().numpy(), a["g"].cpu().numpy().reshape(-1), a["cst"].cpu().numpy()


class NodeEpoch:
    """The C3 epoch on a one-process node (hbtc_node_*, `--node`): device slot d holds whole
    ciphertexts [first[d], first[d+1]) (hbtc_shard_instances, balanced by share count) resident
    in its HBM; a step enqueues every slot's verification, then every slot's combines of its own
    ciphertexts (hbtc_node_verify_dec_shares_dev / hbtc_node_combine_dec_verified_dev, one host
    thread per device).  No collective: the slots' verdicts and combined points are disjoint
    slices of the epoch, final where they are computed (one process owns every device)."""

    def __init__(self, node, args, slices):
        self.node = node
        self.ctxs = [node.context(d) for d in range(len(node.devices))]
        self.eps = [Epoch(c, args.n, args.cts, SEED, args.corrupt, args.corrupt_mode, ct_range=slices[d][0],
                          load_keyset=False) for d, c in enumerate(self.ctxs)]
        self.keyset, bad = node.keyset_load(self.eps[0].pk)
        assert bad == 0
        self.t = self.eps[0].t
        self.total = sum(ep.total for ep in self.eps)
        self.m = sum(ep.m for ep in self.eps)
        self.n, self.f = self.eps[0].n, self.eps[0].f
        self.parts = []
        for j in range(N_OUT):
            specs = [{"offsets": ep.offsets, "d_H_c96": ep.d["H"], "d_w_c96": ep.d["w"], "d_idx": ep.d["idx"],
                      "d_items": ep.d["shares"], "d_status": ep.ptr(j, "status"), "d_out": ep.ptr(j, "g"),
                      "d_inst_status": ep.ptr(j, "cst")} if ep.m else {} for ep in self.eps]
            self.parts.append(node.parts(specs))
        self.cur = 0

    def step(self, ctx=None):
        self.cur = (self.cur + 1) % N_OUT
        for ep in self.eps:
            ep.cur = self.cur
        parts, _ = self.parts[self.cur]
        self.node.verify_dec_shares_dev(self.keyset, parts)
        self.node.combine_dec_verified_dev(parts, self.t)

    def check(self, ctx, args):
        self.node.sync()
        st, g, cst = [], [], []
        for c, ep in zip(self.ctxs, self.eps):
            if ep.m:
                a, b, x = ep.results(c)
                st.append(a)
                g.append(b)
                cst.append(x)
        st, g, cst = np.concatenate(st), np.concatenate(g), np.concatenate(cst)
        expected = np.concatenate([ep.expected for ep in self.eps])
        want, _ = ctx.g1_mul(G1_GEN, scalars_bytes(_all_master_r(args, self.eps[0])))
        return (int((st != expected).sum()), bool((cst == 0).all() and bytes(g) == bytes(want)),
                int((st == N.ACCEPT).sum()))


def timed_node(nep, steps, warmup):
    """timed() for the node: W untimed steps, then K steps bracketed by node-wide syncs."""
    c0 = nep.ctxs[0]
    c0.timing_enable(True)
    for _ in range(warmup):
        nep.step()
    nep.node.sync()
    c0.timing_reset()
    t0 = time.perf_counter()
    for _ in range(steps):
        nep.step()
    nep.node.sync()
    return time.perf_counter() - t0


def cpu_baseline(ep, budget_s):
    """The oracle (threshold_crypto restatement) on a bounded sample of the same workload: per
    share the reference's verify_decryption_share = hash_g1_g2(u, v) + two full pairings, plus
    the serde decode (subgroup check) of the share.  C restatement when built (oracle/c), else
    the Python restatement across a process pool."""
    try:
        from oracle.cbaseline import run_dec_share_baseline
        return run_dec_share_baseline(ep, budget_s)
    except ImportError:
        pass
    from oracle.pybaseline import run_dec_share_baseline
    return run_dec_share_baseline(ep, budget_s)


def rank_seed(rank):
    """Seed of a rank's epoch under --scaling weak: ranks verify disjoint, independently
    generated epochs (no shared state besides the read-only key set)."""
    return SEED + 7919 * rank


def max_over_ranks(elapsed, dist, device=None):
    """The job's time: barrier, then the MAX of the ranks' timed regions (all-reduce on the
    process group's backend: host tensor for gloo, device tensor for RCCL)."""
    if dist is None:
        return elapsed
    import torch
    dist.barrier()
    tt = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


PROFILE_ROUND = "r06"


def profile_dir(args, world):
    """The committed rocprofv3 summaries of this bench command's workload (kernel trace + PMC
    passes, tools/profile.sh): profiles/<round>/bench_<cts>ct_<bits>b[_<world>r], or None."""
    tag = "bench_%dct_%db" % (args.cts, args.rlc_bits) + ("_%dr" % world if world > 1 else "")
    if args.corrupt_mode != "uniform" or args.mode != "rlc" or args.n != 1000:
        return None
    d = os.path.join("profiles", PROFILE_ROUND, tag)
    return d if os.path.exists(os.path.join(ROOT, d, "kt_kernel_stats.csv")) else None


def rocprof_avg_ms(prof_dir, kernel):
    """Average duration (ms) of `kernel`'s FULL-SIZE launches in the committed kernel trace
    (kt_launches.csv: the largest grid only -- a cold key set's probe pass is a smaller launch of
    the same kernel), with the launch count; else the --stats table's average over all launches."""
    import csv
    p = os.path.join(ROOT, prof_dir, "kt_launches.csv")
    if os.path.exists(p):
        with open(p, newline="") as fh:
            rows = [r for r in csv.DictReader(fh) if r["kernel"].endswith("hbtc::" + kernel)]
        if rows:
            g = max(int(r["grid_x"]) for r in rows)
            d = [int(r["duration_ns"]) for r in rows if int(r["grid_x"]) == g]
            return round(sum(d) / len(d) / 1e6, 3), len(d), "kt_launches.csv (full-size launches, grid %d)" % g
    p = os.path.join(ROOT, prof_dir, "kt_kernel_stats.csv")
    if not os.path.exists(p):
        return None, 0, None
    with open(p, newline="") as fh:
        for row in csv.DictReader(fh):
            name = row["Name"].split("(")[0]
            if name.endswith("hbtc::" + kernel):
                return round(float(row["AverageNs"]) / 1e6, 3), int(row["Calls"]), "kt_kernel_stats.csv (all launches)"
    return None, 0, None


N_OUT = 6  # output sets rotated per step (Epoch.step): four epochs in flight + two gathers
# diagnostics of the merge's cost (never set by the driver): HBTC_BENCH_SKIP = comma list of
# wait (output-set reuse wait), order (gather after the verification), gather (the collectives)
DIAG_SKIP = set(filter(None, os.environ.get("HBTC_BENCH_SKIP", "").split(",")))

FAMS = ["dec_verify", "rlc_items", "chk_tiles", "chk_tiles_w", "chk_halves", "chk_halves_w", "chk_subs", "chk_subs_w",
        "chk_split1", "chk_split2", "chk_split3", "chk_leaves", "rlc_finalize", "lagrange", "comb_decode",
        "comb_digits", "combine", "prepare"]


def timed(ctx, ep, steps, warmup, dist=None, gather=None, sync_all=None):
    """W untimed steps, then exactly K steps bracketed by barrier + device syncs."""
    host_t = [0.0, 0.0, 0.0]

    def run():
        t = time.perf_counter()
        if gather:
            gather.before_step(ctx)
        t1 = time.perf_counter()
        ep.step(ctx)
        t2 = time.perf_counter()
        if gather:
            gather.after_step(ctx)
        t3 = time.perf_counter()
        host_t[0] += t1 - t
        host_t[1] += t2 - t1
        host_t[2] += t3 - t2

    def fence():
        ctx.sync()
        if sync_all:
            sync_all()

    ctx.timing_enable(True)
    for _ in range(warmup):
        run()
    fence()
    ctx.timing_reset()
    if dist:
        dist.barrier()
    fence()
    host_t[:] = [0.0, 0.0, 0.0]
    t0 = time.perf_counter()
    for _ in range(steps):
        run()
    fence()
    dt = time.perf_counter() - t0
    if DIAG_SKIP or os.environ.get("HBTC_BENCH_HOSTT"):
        print("host ms per step: before %.2f  step %.2f  after %.2f; %.2f ms per step in all"
              % (tuple(1e3 * x / steps for x in host_t) + (1e3 * dt / steps,)), file=sys.stderr, flush=True)
    return dt


def rlc_width_line(ctx, ep, args, bits):
    """The headline epoch with the other RLC scalar width (hbtc_set_rlc_bits): 64-bit scalars
    give <= 2^-64 per group check, 128-bit <= 2^-128 (DESIGN.md §4 "Soundness").  Same epoch,
    same steps, decisions and combines checked against the construction."""
    ctx.set_rlc_bits(bits)
    try:
        elapsed = timed(ctx, ep, args.steps, args.warmup)
        per = {f: round(ctx.timing_read(f)[0] / args.steps, 3) for f in FAMS if ctx.timing_read(f)[1]}
        mism, comb_ok, _ = ep.check(ctx)
    finally:
        ctx.set_rlc_bits(args.rlc_bits)
    if mism or not comb_ok:
        raise SystemExit("rlc%d: results differ from the construction (%d mismatches, combine %s)"
                         % (bits, mism, comb_ok))
    return {"value": round(ep.total * args.steps / elapsed, 1), "unit": "shares/s",
            "ms_per_step": round(elapsed / args.steps * 1e3, 3), "steps": args.steps, "rlc_bits": bits,
            "soundness_per_group_check": "2^-%d" % bits, "results_ok": True,
            "kernel_event_spans_ms_per_step": per}


def host_buffer_line(ctx, ep, steps, warmup=2):
    """The epoch through the pipelined host-buffer entry point (what an FFI caller holding wire
    bytes does, hbtc_dec_epoch_submit / hbtc_wait): per epoch, the compressed shares, indices,
    H and w go from host memory through pinned staging to the device, the shares are verified,
    the first t verified shares of every ciphertext combined, and statuses and points come back
    to host memory -- all inside the timed region.  Up to four epochs are in flight (hbbft's
    current epoch + max_future_epochs = 3), so epoch k's copies overlap the others' kernels."""
    from collections import deque
    sh = ep.host_shares.reshape(-1)
    n_sets = 6
    outs = [None] * n_sets
    inflight = deque()

    def run(k):
        if len(inflight) == 4:
            inflight.popleft().wait()
        p = ctx.dec_epoch_submit(ep.keyset, ep.H, ep.w, ep.offsets, ep.idx, sh, ep.t, outs[k % n_sets])
        outs[k % n_sets] = p.outs
        inflight.append(p)
        return p

    for k in range(warmup):
        run(k)
    while inflight:
        inflight.popleft().wait()
    t0 = time.perf_counter()
    last = None
    for k in range(steps):
        last = run(warmup + k)
    while inflight:
        inflight.popleft().wait()
    elapsed = time.perf_counter() - t0
    st, g, cst = last.outs
    ok = bool((st[:ep.total] == ep.expected).all() and (cst[:ep.m] == 0).all()
              and g[:ep.m].tobytes() == bytes(ep.want_g(ctx)))
    return {"value": round(ep.total * steps / elapsed, 1), "unit": "shares/s",
            "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps, "warmup": warmup,
            "results_ok": ok,
            "path": "hbtc_dec_epoch_submit + hbtc_wait (host buffers, up to 4 epochs in flight: pinned "
                    "staging, H2D of compressed shares / idx / H / w, verification, combine of the first t "
                    "verified shares, D2H of statuses and points inside the timed region)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--validators", dest="n", type=int, default=1000, help="validators N (f = (N-1)/3)")
    ap.add_argument("--cts", type=int, default=1000,
                    help="ciphertexts per epoch (strong: of the whole job; weak: per GPU)")
    ap.add_argument("--scaling", choices=["strong", "weak"], default="strong")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the adversarial / host-buffer lines")
    ap.add_argument("--mode", choices=["rlc", "per_share"], default="rlc",
                    help="rlc: batched random-linear-combination checks with exact fallback "
                         "(default); per_share: one pairing check per share")
    ap.add_argument("--rlc-bits", type=int, choices=[64, 128], default=None,
                    help="RLC scalar size (hbtc_set_rlc_bits): soundness 2^-128 (the library default, "
                         "SURVEY.md §7 step 5) or 2^-64 per group check")
    ap.add_argument("--corrupt", type=float, default=0.01, help="fraction of wrong shares")
    ap.add_argument("--corrupt-mode", choices=["uniform", "senders"], default="uniform")
    ap.add_argument("--node", action="store_true",
                    help="with --gpus N > 1 in ONE process (no torchrun): a multi-device node "
                         "(hbtc_node_*_dev) splits the epoch by whole ciphertexts over N GPUs; no "
                         "collective, no torch.distributed")
    ap.add_argument("--slots", default=None,
                    help="--node device slots, e.g. 0,0 (two contexts on GPU 0: a rehearsal)")
    ap.add_argument("--force-dist", action="store_true",
                    help="initialise torch.distributed and run the strong-scaling merge even at "
                         "WORLD_SIZE 1 (torchrun --nproc-per-node 1: exercises the RCCL path on one GPU)")
    ap.add_argument("--backend", choices=["nccl", "gloo"], default="nccl",
                    help="process-group backend of the merge (nccl = RCCL over xGMI; gloo only to "
                         "rehearse the sharded path with several ranks on one GPU)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.node and world == 1 and (args.gpus > 1 or args.slots):
        return node_main(args)
    use_dist = world > 1 or args.force_dist
    strong = args.scaling == "strong" and use_dist
    dist, torch, dev = None, None, None
    if use_dist:
        import torch
        import torch.distributed as dist
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dev = torch.device("cuda", local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    ctx = N.Context(local)
    t0 = time.time()
    ctx.set_verify_mode(N.MODE_RLC if args.mode == "rlc" else N.MODE_PER_SHARE)
    if args.rlc_bits is None:
        args.rlc_bits = ctx.rlc_bits()  # the library default
    ctx.set_rlc_bits(args.rlc_bits)
    gather, slices = None, None
    if strong:
        from hbbft_amd import shard
        offsets_all = np.arange(0, args.n * args.cts + 1, args.n, dtype=np.uint32)
        slices = shard.instance_slices(world, offsets_all)

        def out_alloc(nbytes, i32):
            tns = torch.zeros(nbytes // 4 if i32 else nbytes, dtype=torch.int32 if i32 else torch.uint8,
                              device=dev)
            return ctypes.c_void_p(tns.data_ptr()), tns
        ep = Epoch(ctx, args.n, args.cts, SEED, args.corrupt, args.corrupt_mode,
                   ct_range=slices[rank][0], out_alloc=out_alloc)
        gather = StrongGather(ep, dist, slices, torch)
    else:
        ep = Epoch(ctx, args.n, args.cts, SEED if world == 1 else rank_seed(rank), args.corrupt,
                   args.corrupt_mode)
    log("rank %d: setup %.1fs (%d shares)" % (rank, time.time() - t0, ep.total))

    elapsed = timed(ctx, ep, args.steps, args.warmup, dist, gather,
                    torch.cuda.synchronize if torch else None)
    elapsed = max_over_ranks(elapsed, dist, dev if args.backend == "nccl" else None)
    breakdown = {f: ctx.timing_read(f) for f in FAMS}
    leaves = ctx.rlc_last_leaves() if args.mode == "rlc" else ep.total
    # the same epoch once more with nothing else in flight (after the timed region): the dominant
    # kernel's duration on an otherwise idle chip, beside its pipelined duration above (where
    # the other lanes' check levels and combines share the CUs with it)
    iso, iso_wall = {}, None
    if gather is None:
        ctx.sync()
        ctx.timing_reset()
        a = time.perf_counter()
        ep.step(ctx)
        ctx.sync()
        iso_wall = time.perf_counter() - a
        iso = {f: ctx.timing_read(f) for f in FAMS}
    if strong and "gather" in DIAG_SKIP:
        mism, comb_ok, n_acc = ep.check(ctx)  # diagnostics without the collectives: local check
    elif strong:
        # the merged whole epoch on every rank, against the whole epoch's construction
        st, g, cst = gather.merged()
        expected = np.concatenate([np.asarray(x) for x in _all_expected(dist, ep, torch, dev, slices)])
        want, _ = ctx.g1_mul(G1_GEN, scalars_bytes(_all_master_r(args, ep)))
        mism = int((st != expected).sum())
        comb_ok = bool((cst == 0).all() and bytes(g) == bytes(want))
        n_acc = int((st == N.ACCEPT).sum())
    else:
        mism, comb_ok, n_acc = ep.check(ctx)
    log("rank %d: %.3fs for %d steps; kernel ms/step %s; leaves %d; mismatches %d, combine ok %s"
        % (rank, elapsed, args.steps,
           {f: round(breakdown[f][0] / args.steps, 1) for f in FAMS if breakdown[f][1]}, leaves,
           mism, comb_ok))
    if mism or not comb_ok:
        raise SystemExit("rank %d: results differ from the construction (%d mismatches, combine %s)"
                         % (rank, mism, comb_ok))

    job_shares = args.n * args.cts * (1 if args.scaling == "strong" else world)
    job_cts = args.cts * (1 if args.scaling == "strong" else world)
    value = job_shares * args.steps / elapsed
    combines = job_cts * args.steps / elapsed
    consts = json.load(open(os.path.join(ROOT, "bench", "roofline_constants.json")))
    n_tiles = ep.m * ((ep.n + 63) // 64)
    sched = ctx.check_schedule_for(n_tiles)
    kname = kernel_names(sched)
    paired = sched != N.CHECK_PLAIN_FIRST
    # algorithmic Fqm per launch of each kernel family (tools/fqm_count.cpp)
    fqm_per_launch = {
        "dec_verify": consts["dec_share"]["total"] * ep.total,
        "rlc_items": consts["rlc_item" if args.rlc_bits == 64 else "rlc_item_128"] * ep.total,
        # the tile level: the plain 2-pair check of every tile, plus (paired schedules) its
        # weighted check in the same launch (serial Fqm count of one check; the location search
        # and the cooperative form's extra lane work are not counted)
        "chk_tiles": consts["rlc_group_check"] * n_tiles * (2 if paired else 1),
        "chk_leaves": consts["dec_share"]["total"] * leaves,
        "combine": consts.get("g1_msm_combine", 0) * ep.m,
    }
    per_step = {f: round(breakdown[f][0] / args.steps, 3) for f in FAMS if breakdown[f][1]}
    # The dominant kernel is chosen among the main-stream (critical-path) families: the
    # combine runs concurrently on its own stream, so its event span includes the time it
    # shares the CUs with the verify chain and is not a launch duration.
    main_stream = ("dec_verify", "rlc_items", "chk_tiles", "chk_leaves")
    dom = max((f for f in main_stream if breakdown[f][1]), key=lambda f: breakdown[f][0])
    dom_avg_s = breakdown[dom][0] / breakdown[dom][1] / 1e3
    achieved = fqm_per_launch[dom] / dom_avg_s * consts["mad_u64_u32_per_fqm"] / 1e12
    # rocprofv3 kernel trace + PMC passes of THIS workload (tools/profile.sh -> tools/
    # pmc_summary.py), committed under profiles/: separate FETCH_SIZE / WRITE_SIZE / SQ passes,
    # FETCH_SIZE doubled per the gfx950 note.  A workload without a committed profile reports
    # null rather than another workload's figures.
    traffic, pmc, rocprof_ms, rocprof_n, rocprof_src = None, {}, None, 0, None
    valu_insts, pmc_parts = None, None
    prof_dir = profile_dir(args, world)
    if prof_dir:
        summ_path = os.path.join(ROOT, prof_dir, "pmc_summary.json")
        # a family launched as two kernels (the item pass: decode, then the scalar half) is priced
        # by the sum of its kernels' launches, like the HIP-event span that covers both
        parts = KERNEL_PARTS.get(dom, (kname[dom],))
        if os.path.exists(summ_path):
            summ = json.load(open(summ_path))
            found = [summ.get("hbtc::" + k) or summ.get("void hbtc::" + k) for k in parts]
            found = [f for f in found if f]
            pmc = found[-1] if found else {}
            if found and all("hbm_read_bytes" in f and "hbm_write_bytes" in f for f in found):
                traffic = sum(f["hbm_read_bytes"] + f["hbm_write_bytes"] for f in found)
            vi = [f.get("counters_mean_per_dispatch", {}).get("SQ_INSTS_VALU") for f in found]
            if found and all(v is not None for v in vi):
                valu_insts = sum(vi)
            pmc_parts = {k: {x: f.get(x) for x in ("grid", "full_size_dispatches", "dispatches", "vgpr",
                                                    "scratch_bytes_per_lane", "valu_busy", "hbm_read_bytes",
                                                    "hbm_write_bytes")}
                         for k, f in zip(parts, found)}
        avgs = [rocprof_avg_ms(prof_dir, k) for k in parts]
        avgs = [a for a in avgs if a[0] is not None]
        if avgs:
            rocprof_ms = round(sum(a[0] for a in avgs), 3)
            rocprof_n = min(a[1] for a in avgs)
            rocprof_src = "; ".join("%s: %s" % (k, a[2]) for k, a in zip(parts, avgs))
    if strong:
        coll = ("RCCL (nccl backend) all-gather over xGMI" if args.backend == "nccl"
                else "gloo all-gather of host copies (rehearsal, not the product merge)")
        par = ("strong: one epoch sharded by whole ciphertexts over %d rank(s), one process per GPU "
               "(hbtc_shard_instances), %s of statuses + combined points" % (world, coll))
    elif world > 1:
        par = "weak: an independent epoch per GPU (%d GPUs), no collective" % world
    else:
        par = "1 GPU"
    out = {
        "metric": "verified BLS12-381 shares/sec (whole node) at N=1000; combines/sec",
        "value": round(value, 1),
        "unit": "shares/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong" if args.scaling == "strong" else "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery limbs)",
        "data": "synthetic (seeded key set, shares generated on device; %s + 8 bad encodings)"
                % ("%g%% wrong shares" % (100 * args.corrupt) if args.corrupt_mode == "uniform"
                   else "f = %d Byzantine senders send wrong shares on every ciphertext" % ep.f),
        "config": {"workload": "C3 HoneyBadger epoch: %d ciphertexts x %d DecryptionShares verified + %d G1 combines (t=%d)%s"
                   % (job_cts, args.n, job_cts, ep.t, "" if args.scaling == "strong" else " per GPU"),
                   "N": args.n, "f": ep.f, "t": ep.t, "ciphertexts": job_cts,
                   "shares_per_step": job_shares, "parallelism": par},
        "combines_per_s": round(combines, 1),
        "accepted_per_step": n_acc,
        "mode": args.mode,
        "rlc_bits": args.rlc_bits,
        "check_schedule": SCHED_NAME[sched],
        "exact_single_share_checks_per_step_rank0": leaves,
        "kernel_event_spans_ms_per_step_rank0": per_step,
        "isolated_epoch": ({"ms": round(iso_wall * 1e3, 3),
                            "spans_ms": {f: round(v[0], 3) for f, v in iso.items() if v[1]},
                            "note": "one more epoch after the timed region with nothing else in flight: its "
                                    "wall time is the lane's chain latency (items -> check levels -> "
                                    "combine); ms_per_step below it means the four lanes overlap"}
                           if iso_wall else None),
        "kernel_event_spans_note": ("HIP-event spans per kernel family on the library's streams, summed "
                                    "per step: the four verification lanes and the preparation stream "
                                    "overlap, so the spans add up to more than ms_per_step; kernel "
                                    "durations are roofline.rocprof_avg_ms_per_launch (rocprofv3)"),
        "roofline": {
            "bound": "valu-int (v_mad_u64_u32)",
            "kernel": " + ".join(KERNEL_PARTS.get(dom, (kname[dom],))),
            "achieved": round(achieved, 3),
            "peak": MAD_U64_PEAK / 1e12,
            "peak_source": MAD_U64_PEAK_NOTE,
            "unit": "T mad_u64_u32/s",
            "frac": round(achieved / (MAD_U64_PEAK / 1e12), 4),
            "traffic": traffic,
            "traffic_unit": "bytes per full-size launch (HBM read + write, rocprofv3 PMC; FETCH_SIZE x2 per "
                            "the gfx950 note), summed over the family's kernels",
            "fqm_per_launch": fqm_per_launch[dom],
            "kernel_ms_per_launch": round(dom_avg_s * 1e3, 3),
            "kernel_ms_per_launch_source": "HIP events on the kernel's stream, this run (the span can "
                                           "include time the kernel shares the CUs with other lanes)",
            "rocprof_avg_ms_per_launch": rocprof_ms,
            "rocprof_launches_averaged": rocprof_n,
            "rocprof_source": rocprof_src,
            "frac_at_rocprof_duration": (round(fqm_per_launch[dom] * consts["mad_u64_u32_per_fqm"]
                                               / (rocprof_ms * 1e-3) / MAD_U64_PEAK, 4) if rocprof_ms else None),
            "profile_dir": prof_dir,
            "kernel_ms_per_launch_isolated": (round(iso[dom][0] / iso[dom][1], 3) if iso.get(dom, (0, 0))[1]
                                              else None),
            "frac_isolated": (round(fqm_per_launch[dom] * consts["mad_u64_u32_per_fqm"]
                                    / (iso[dom][0] / iso[dom][1] * 1e-3) / MAD_U64_PEAK, 4)
                              if iso.get(dom, (0, 0))[1] else None),
            "isolated_note": "one extra epoch after the timed region with no other epoch in flight",
            "pmc": pmc_parts,
            "pmc_note": ("per kernel: means over the full-size dispatches only (grid = the kernel's "
                         "largest in the pass; a key set's probe pass is excluded), tools/pmc_summary.py"),
            "valu_wave_insts_per_launch": valu_insts,
            "valu_wave_insts_per_wave_mad": (round(valu_insts / (fqm_per_launch[dom]
                                                                * consts["mad_u64_u32_per_fqm"] / 64), 3)
                                             if valu_insts else None),
        },
    }
    if world == 1 and not args.no_extra:
        # the other RLC width on the same epoch (SURVEY.md §7 step 5 specifies 128-bit scalars;
        # the headline runs the library default)
        alt = 64 if args.rlc_bits == 128 else 128
        out["rlc%d" % alt] = rlc_width_line(ctx, ep, args, alt)
        out["host_buffers"] = host_buffer_line(ctx, ep, args.steps, min(args.warmup, 2))
        if args.corrupt_mode == "uniform":
            out["adversarial"] = adversarial_line(ctx, args, ep)
    if rank == 0 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(ep, args.cpu_budget)
        except Exception as e:  # the baseline is reported, never the product path
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


def node_main(args):
    """--node: the epoch on a one-process multi-device node (NodeEpoch)."""
    from hbbft_amd import shard
    slots = [int(x) for x in args.slots.split(",")] if args.slots else list(range(args.gpus))
    ctx = N.Context(slots[0])
    node = N.Node(slots)
    node.set_verify_mode(N.MODE_RLC if args.mode == "rlc" else N.MODE_PER_SHARE)
    node.set_rlc_bits(args.rlc_bits)
    offsets_all = np.arange(0, args.n * args.cts + 1, args.n, dtype=np.uint32)
    slices = shard.instance_slices(len(slots), offsets_all)
    t0 = time.time()
    nep = NodeEpoch(node, args, slices)
    log("node: setup %.1fs (%d shares over %d slots)" % (time.time() - t0, nep.total, len(slots)))
    elapsed = timed_node(nep, args.steps, args.warmup)
    mism, comb_ok, n_acc = nep.check(ctx, args)
    per = {f: round(nep.ctxs[0].timing_read(f)[0] / args.steps, 3) for f in FAMS
           if nep.ctxs[0].timing_read(f)[1]}
    log("node: %.3fs for %d steps; slot-0 event spans ms/step %s; mismatches %d, combine ok %s"
        % (elapsed, args.steps, per, mism, comb_ok))
    if mism or not comb_ok:
        raise SystemExit("node: results differ from the construction (%d mismatches, combine %s)" % (mism, comb_ok))
    n_gpus = len(set(slots))
    out = {
        "metric": "verified BLS12-381 shares/sec (whole node) at N=1000; combines/sec",
        "value": round(nep.total * args.steps / elapsed, 1), "unit": "shares/s", "n_gpus": n_gpus,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery limbs)",
        "data": "synthetic (seeded key set, shares generated on device; %s + 8 bad encodings)"
                % ("%g%% wrong shares" % (100 * args.corrupt) if args.corrupt_mode == "uniform"
                   else "f = %d Byzantine senders send wrong shares on every ciphertext" % nep.f),
        "config": {"workload": "C3 HoneyBadger epoch: %d ciphertexts x %d DecryptionShares verified + %d G1 "
                               "combines (t=%d)" % (args.cts, args.n, args.cts, nep.t),
                   "N": args.n, "f": nep.f, "t": nep.t, "ciphertexts": args.cts,
                   "shares_per_step": nep.total,
                   "parallelism": "node: one process, %d device slot(s) on %d GPU(s) (hbtc_node_*_dev), whole "
                                  "ciphertexts per slot (hbtc_shard_instances); no collective (disjoint "
                                  "outputs)" % (len(slots), n_gpus)},
        "combines_per_s": round(args.cts * args.steps / elapsed, 1),
        "accepted_per_step": n_acc, "mode": args.mode,
        "kernel_event_spans_ms_per_step_slot0": per,
    }
    print(json.dumps(out), flush=True)
    node.close()
    ctx.close()


def _all_expected(dist, ep, torch, dev, slices):
    """Every rank's expected statuses (construction), gathered over the job (check only)."""
    from hbbft_amd import shard
    loc = torch.from_numpy(ep.expected).to(dev)
    return [shard.gather_slices(dist, loc, [hi - lo for _, (lo, hi) in slices]).cpu().numpy()]


def _all_master_r(args, ep):
    """master_sk * r_k of every ciphertext of the whole epoch (r_k derives from (seed, k))."""
    return [ep.master_sk * random.Random(SEED * 1000003 + k).randrange(1, R) % R
            for k in range(args.cts)]


def adversarial_line(ctx, args, base):
    """The same configuration under BFT's worst case: f = 333 Byzantine senders send wrong
    shares on every ciphertext (33 % of all shares, concentrated by sender).  A fresh key set,
    so the first epoch's call starts with a probe pass over its first ciphertexts that finds the
    liars (reported as first_epoch_ms); the timed steps then run with the liars tracked
    (hbtc_set_sender_tracking, default on)."""
    base.free(ctx)
    ep = Epoch(ctx, args.n, args.cts, SEED, 0.0, "senders")
    ctx.sync()
    t0 = time.perf_counter()
    ep.step(ctx)
    ctx.sync()
    first = time.perf_counter() - t0
    first_leaves = ctx.rlc_last_leaves() if args.mode == "rlc" else ep.total
    steps = max(1, min(args.steps, 6))
    elapsed = timed(ctx, ep, steps, 1)
    per = {f: round(ctx.timing_read(f)[0] / steps, 3) for f in FAMS if ctx.timing_read(f)[1]}
    leaves = ctx.rlc_last_leaves() if args.mode == "rlc" else ep.total
    mism, comb_ok, n_acc = ep.check(ctx)
    if mism or not comb_ok:
        raise SystemExit("adversarial: results differ from the construction (%d mismatches, combine %s)"
                         % (mism, comb_ok))
    ep.free(ctx)
    return {"value": round(ep.total * steps / elapsed, 1), "unit": "shares/s",
            "ms_per_step": round(elapsed / steps * 1e3, 3), "steps": steps,
            "first_epoch_ms": round(first * 1e3, 3), "first_epoch_leaves": first_leaves,
            "data": "f = %d Byzantine senders send wrong shares on every ciphertext (%d of %d shares) + 8 bad encodings"
                    % (ep.f, ep.f * ep.m, ep.total),
            "accepted_per_step": n_acc, "exact_single_share_checks_per_step": leaves,
            "kernel_event_spans_ms_per_step": per,
            "kernel_event_spans_note": "HIP-event spans: they include queueing behind the other lanes' kernels (k_rlc_finalize runs ~0.02 ms in rocprofv3 traces)"}


if __name__ == "__main__":
    main()
