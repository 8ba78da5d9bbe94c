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

Multi-GPU (weak scaling): one process per GPU (torch.distributed.run), each rank verifies its
own epoch shard of 1000 ciphertexts (shards are independent, SURVEY.md §8e: no data-path
collective); gloo carries the barrier and the max-over-ranks time only.

Prints ONE JSON line on rank 0 (contract in the task statement), with "roofline" (the longest
critical-path kernel of the default RLC mode; Fqm counted by tools/fqm_count.cpp ->
bench/roofline_constants.json; HBM traffic from the committed PMC passes) and
"cpu_baseline" (the oracle's threshold_crypto restatement timed on this host).
"""
import argparse
import json
import os
import random
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from hbbft_amd import _native as N  # noqa: E402

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
G1_GEN = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G2_GEN = bytes.fromhex("93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
                       "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")
SEED = 0x6862626674
# measured v_mad_u64_u32 lane-op throughput on MI355X (tools/microbench/intmul.hip,
# profiles/r01_intmul_microbench.txt): the VALU integer-multiply roofline of the Fqm kernels
MAD_U64_PEAK = 29.51e12
# timing family -> kernel (hbtc_api.hip timed() families, rocprofv3 names)
KERNEL_NAME = {"dec_verify": "k_dec_verify", "rlc_items": "k_rlc_items",
               "chk_tiles": "k_chk_tiles", "chk_subs": "k_chk_subs", "chk_leaves": "k_chk_leaves"}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def scalars_bytes(vals):
    return np.frombuffer(b"".join(int(v).to_bytes(32, "little") for v in vals), dtype=np.uint8).copy()


class Epoch:
    """Synthetic C3 epoch for one rank, generated on the GPU with the library's batched scalar
    multiplication (setup, outside the timed region)."""

    def __init__(self, ctx, n, n_ct, seed, corrupt_frac=0.01):
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
        pk, st = ctx.g1_mul(G1_GEN, scalars_bytes(sks))
        assert not st.any()
        self.keyset, bad = ctx.keyset_load(pk)
        assert bad == 0
        rs = [rng.randrange(1, R) for _ in range(n_ct)]
        hs = [rng.randrange(1, R) for _ in range(n_ct)]
        self.rs = rs
        H, _ = ctx.g2_mul(G2_GEN, scalars_bytes(hs))
        w, _ = ctx.g2_mul(G2_GEN, scalars_bytes([r * h % R for r, h in zip(rs, hs)]))
        u, _ = ctx.g1_mul(G1_GEN, scalars_bytes(rs))
        self.pk_bytes = [bytes(pk[48 * i:48 * i + 48]) for i in range(n)]
        self.u_bytes = [bytes(u[48 * k:48 * k + 48]) for k in range(n_ct)]
        self.w_bytes = [bytes(w[96 * k:96 * k + 96]) for k in range(n_ct)]
        total = n * n_ct
        scal = [sks[i] * rs[k] % R for k in range(n_ct) for i in range(n)]
        # corruption: wrong shares (valid points) and bad encodings anywhere; the combine takes
        # the first t VERIFIED shares of every ciphertext, as hbbft does
        self.expected = np.zeros(total, np.int32)
        n_bad = int(total * corrupt_frac)
        cand = rng.sample(range(total), min(total, n_bad + 8))
        wrong, enc = cand[:n_bad], cand[n_bad:n_bad + 8]
        for j in wrong:
            scal[j] = (scal[j] + 1) % R
            self.expected[j] = N.REJECT
        shares, st = ctx.g1_mul(G1_GEN, scalars_bytes(scal))
        assert not st.any()
        shares = shares.reshape(total, 48)
        for j in enc:
            shares[j, 0] &= 0x7F  # clear the compression flag: pairing 0.14 rejects it
            self.expected[j] = N.DECODE_ERR
        self.offsets = np.arange(0, total + 1, n, dtype=np.uint32)
        idx = np.tile(np.arange(n, dtype=np.uint32), n_ct)
        # resident device copies
        self.d = {}
        for name, arr in (("H", H), ("w", w), ("idx", idx), ("shares", shares.reshape(-1))):
            p = ctx.dev_alloc(arr.nbytes)
            ctx.dev_upload(p, arr)
            self.d[name] = p
        # two sets of outputs, alternated per step: epoch k+1's verification writes one status
        # array while epoch k's combine still reads the other (hbtc.h ordering rules)
        for j in range(2):
            self.d["status%d" % j] = ctx.dev_alloc(4 * total)
            self.d["g%d" % j] = ctx.dev_alloc(48 * n_ct)
            self.d["cst%d" % j] = ctx.dev_alloc(4 * n_ct)
        self.cur = 0
        self.total = total
        self.host_shares = shares

    def step(self, ctx):
        """One epoch: the 10^6 share checks, then the 1000 combines of the first t VERIFIED
        shares of every ciphertext (PublicKeySet::decrypt over ThresholdDecryption's verified
        share map, td.rs:184).  The combines run on the library's combine stream behind this
        epoch's verification, so they overlap the NEXT epoch's verification (pipelined epochs);
        the timed region ends when the last combine is done."""
        lib, h, d = ctx.lib, ctx.h, self.d
        self.cur ^= 1
        j = self.cur
        off = N._ptr(self.offsets)
        ctx._check(lib.hbtc_verify_dec_shares_dev(h, self.keyset, self.n_ct, d["H"], d["w"], off,
                                                  d["idx"], d["shares"], d["status%d" % j]),
                   "verify_dec_shares_dev")
        ctx._check(lib.hbtc_combine_dec_verified_dev(h, self.n_ct, off, d["idx"], d["shares"],
                                                     d["status%d" % j], self.t, d["g%d" % j],
                                                     d["cst%d" % j]),
                   "combine_dec_verified_dev")

    def check(self, ctx):
        j = self.cur  # the last step's outputs
        st = np.empty(self.total, np.int32)
        ctx.dev_download(st, self.d["status%d" % j])
        mism = int((st != self.expected).sum())
        g = np.empty(48 * self.n_ct, np.uint8)
        ctx.dev_download(g, self.d["g%d" % j])
        cst = np.empty(self.n_ct, np.int32)
        ctx.dev_download(cst, self.d["cst%d" % j])
        want, _ = ctx.g1_mul(G1_GEN, scalars_bytes([self.master_sk * r % R for r in self.rs]))
        comb_ok = bool((cst == 0).all() and bytes(g) == bytes(want))
        return mism, comb_ok, int((st == N.ACCEPT).sum())


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
    """Seed of a rank's epoch shard: ranks verify disjoint, independently generated epochs
    (weak scaling, SURVEY.md §8e: no shared state besides the read-only key set)."""
    return SEED + 7919 * rank


def max_over_ranks(elapsed, dist):
    """The job's time: barrier, then the MAX of the ranks' timed regions (gloo all-reduce)."""
    if dist is None:
        return elapsed
    import torch
    dist.barrier()
    tt = torch.tensor([elapsed], dtype=torch.float64)
    dist.all_reduce(tt, op=dist.ReduceOp.MAX)
    return float(tt.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=1000, help="validators N (f = (N-1)/3)")
    ap.add_argument("--cts", type=int, default=1000, help="ciphertexts per epoch per GPU")
    ap.add_argument("--cpu-budget", type=float, default=20.0, help="seconds of CPU baseline")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--mode", choices=["rlc", "per_share"], default="rlc",
                    help="rlc: batched random-linear-combination checks with exact fallback "
                         "(default); per_share: one pairing check per share")
    ap.add_argument("--corrupt", type=float, default=0.01, help="fraction of wrong shares")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    ctx = N.Context(local)
    t0 = time.time()
    ctx.set_verify_mode(N.MODE_RLC if args.mode == "rlc" else N.MODE_PER_SHARE)
    ep = Epoch(ctx, args.n, args.cts, rank_seed(rank), corrupt_frac=args.corrupt)
    log("rank %d: setup %.1fs (%d shares)" % (rank, time.time() - t0, ep.total))

    ctx.timing_enable(True)
    for _ in range(args.warmup):
        ep.step(ctx)
    ctx.sync()
    ctx.timing_reset()
    if dist:
        dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        ep.step(ctx)
    ctx.sync()
    elapsed = time.perf_counter() - t0
    elapsed = max_over_ranks(elapsed, dist)
    fams = ["dec_verify", "rlc_items", "chk_tiles", "chk_subs", "chk_leaves", "rlc_finalize",
            "lagrange", "comb_decode", "comb_digits", "combine", "prepare"]
    breakdown = {f: ctx.timing_read(f) for f in fams}
    leaves = ctx.rlc_last_leaves() if args.mode == "rlc" else ep.total
    mism, comb_ok, n_acc = ep.check(ctx)
    log("rank %d: %.3fs for %d steps; kernel ms/step %s; leaves %d; mismatches %d, combine ok %s"
        % (rank, elapsed, args.steps,
           {f: round(breakdown[f][0] / args.steps, 1) for f in fams if breakdown[f][1]}, leaves,
           mism, comb_ok))
    if mism or not comb_ok:
        raise SystemExit("rank %d: results differ from the construction (%d mismatches, combine %s)"
                         % (rank, mism, comb_ok))

    shares_total = ep.total * world * args.steps
    value = shares_total / elapsed
    combines = args.cts * world * args.steps / elapsed
    consts = json.load(open(os.path.join(ROOT, "bench", "roofline_constants.json")))
    n_tiles = sum((ep.n + 63) // 64 for _ in range(ep.n_ct))
    # algorithmic Fqm per launch of each kernel family (tools/fqm_count.cpp)
    fqm_per_launch = {
        "dec_verify": consts["dec_share"]["total"] * ep.total,
        "rlc_items": consts["rlc_item"] * ep.total,
        # a tile unit = the plain and the weighted 2-pair check (serial Fqm count of one check;
        # the cooperative kernel issues more lane-level work than this)
        "chk_tiles": consts["rlc_group_check"] * 2 * n_tiles,
        "chk_leaves": consts["dec_share"]["total"] * leaves,
        "combine": consts.get("g1_msm_combine", 0) * ep.n_ct,
    }
    per_step = {f: round(breakdown[f][0] / args.steps, 3) for f in fams if breakdown[f][1]}
    # The dominant kernel is chosen among the main-stream (critical-path) families: the
    # combine runs concurrently on its own stream, so its event span includes the time it
    # shares the CUs with the verify chain and is not a launch duration.
    main_stream = ("dec_verify", "rlc_items", "chk_tiles", "chk_leaves")
    dom = max((f for f in main_stream if breakdown[f][1]), key=lambda f: breakdown[f][0])
    dom_avg_s = breakdown[dom][0] / breakdown[dom][1] / 1e3
    achieved = fqm_per_launch[dom] / dom_avg_s * consts["mad_u64_u32_per_fqm"] / 1e12
    # HBM traffic and VALU instruction count of the same kernel from the committed rocprofv3
    # PMC passes of this command (tools/gpu_configs_pmc.sh -> tools/pmc_summary.py): separate
    # FETCH_SIZE / WRITE_SIZE / SQ passes, FETCH_SIZE doubled per the gfx950 note.
    traffic, pmc = None, {}
    pmc_path = os.path.join(ROOT, "profiles", "r02_pmc_summary.json")
    if os.path.exists(pmc_path):
        pmc = json.load(open(pmc_path)).get("hbtc::" + KERNEL_NAME[dom], {})
        if "hbm_read_bytes" in pmc and "hbm_write_bytes" in pmc:
            traffic = pmc["hbm_read_bytes"] + pmc["hbm_write_bytes"]
    out = {
        "metric": "verified BLS12-381 shares/sec (whole node) at N=1000; combines/sec",
        "value": round(value, 1),
        "unit": "shares/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u32 (381-bit Montgomery limbs)",
        "data": "synthetic (seeded key set, shares generated on device; %g%% wrong shares + 8 bad encodings)"
                % (100 * args.corrupt),
        "config": {"workload": "C3 HoneyBadger epoch: %d ciphertexts x %d DecryptionShares verified + %d G1 combines (t=%d) per GPU"
                   % (args.cts, args.n, args.cts, ep.t),
                   "N": args.n, "f": ep.f, "t": ep.t, "ciphertexts_per_gpu": args.cts,
                   "shares_per_step": ep.total * world, "parallelism": "shard ciphertexts over %d GPU(s)" % world},
        "combines_per_s": round(combines, 1),
        "accepted_per_step_rank0": n_acc,
        "mode": args.mode,
        "exact_single_share_checks_per_step": leaves,
        "kernel_ms_per_step": per_step,
        "roofline": {
            "bound": "valu-int (v_mad_u64_u32)",
            "kernel": KERNEL_NAME[dom],
            "achieved": round(achieved, 3),
            "peak": MAD_U64_PEAK / 1e12,
            "unit": "T mad_u64_u32/s",
            "frac": round(achieved / (MAD_U64_PEAK / 1e12), 4),
            "traffic": traffic,
            "traffic_unit": "bytes per launch (HBM read + write, rocprofv3 PMC)",
            "fqm_per_launch": fqm_per_launch[dom],
            "kernel_ms_per_launch": round(dom_avg_s * 1e3, 3),
            "pmc": {k: pmc[k] for k in ("vgpr", "scratch_bytes_per_lane", "valu_busy",
                                        "hbm_read_bytes", "hbm_write_bytes") if k in pmc} or None,
            "valu_insts_per_launch": pmc.get("counters_mean_per_dispatch", {}).get("SQ_INSTS_VALU"),
        },
    }
    if rank == 0 and not args.no_cpu:
        try:
            out["cpu_baseline"] = cpu_baseline(ep, args.cpu_budget)
        except Exception as e:  # the baseline is reported, never the product path
            out["cpu_baseline"] = {"error": repr(e)}
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
