"""Diagnostics: C2 pipelined steps on a context after a prelude of small calls on the same context
(bench_configs.py c1 then c2 measured 22 ms per C2 step against 13.4 alone).  Usage:
  python tools/r04/c2_after.py PRELUDE   with PRELUDE one of
  none | sig1 (one 10-share verify_sig_shares) | sig3 | sig52 | keyset (load + free a key set) |
  lanes3 (three device-resident 10-share calls, shifting the lane rotation) | c1 (bench_c1, 5 calls)"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench_configs as B  # noqa: E402  (sets 16 hardware queues before the first HIP call)
from hbbft_amd import _native as N  # noqa: E402
import numpy as np  # noqa: E402


def main():
    prelude = sys.argv[1]
    ctx = N.Context(0)
    ctx.set_verify_mode(N.MODE_RLC)
    rng = random.Random(5)
    if prelude != "none":
        if prelude == "c1":
            B.ctx_mode[0] = N.MODE_RLC
            B.bench_c1(ctx, 5, 1)
        else:
            n = 10
            master, sks = B.key_shares(rng, n)
            pk, _ = ctx.g1_mul(B.G1_GEN, B.fr_bytes(sks))
            H = N.hash_g2(B.COIN_NONCE)
            sigs, _ = ctx.g2_mul(H, B.fr_bytes(sks))
            ks, _ = ctx.keyset_load(pk)
            idx = np.arange(n, dtype=np.uint32)
            sl = [bytes(sigs[96 * i:96 * i + 96]) for i in range(n)]
            calls = {"sig1": 1, "sig3": 3, "sig3trim": 3, "sig52": 52, "keyset": 0, "lanes3": 0}[prelude]
            for _ in range(calls):
                ctx.verify_sig_shares(ks, [H], [n], idx, sl)
            if prelude == "lanes3":
                d = {k: ctx.dev_alloc(s) for k, s in (("H", 96), ("idx", 4 * n), ("sig", 96 * n), ("st", 4 * n))}
                ctx.dev_upload(d["H"], np.frombuffer(H, np.uint8))
                ctx.dev_upload(d["idx"], idx)
                ctx.dev_upload(d["sig"], np.frombuffer(b"".join(sl), np.uint8))
                off = np.array([0, n], np.uint32)
                for _ in range(3):
                    ctx._check(ctx.lib.hbtc_verify_sig_shares_dev(ctx.h, ks, 1, d["H"], N._ptr(off), d["idx"],
                                                                  d["sig"], d["st"]), "dev")
                ctx.sync()
            ctx.keyset_free(ks)
            if prelude == "sig3trim":
                ctx.trim_workspace()
    t0 = time.time()
    out = B.bench_coins(ctx, "c2", 100, 100, 20, 2)
    # host issue time per step: the same runner, steps timed on the host without a sync
    inp = B.coin_inputs(ctx, 100, 100)
    run = B.CoinRunner(ctx, inp, 100)
    for _ in range(4):
        run.step()
    run.sync()
    host = []
    a0 = time.perf_counter()
    for _ in range(20):
        a = time.perf_counter()
        run.step()
        host.append(time.perf_counter() - a)
    run.sync()
    wall = (time.perf_counter() - a0) / 20
    host.sort()
    print("prelude %-7s c2 %.3f ms per step (%.0f shares/s); rerun %.3f ms per step, host issue median %.3f "
          "max %.3f ms  [%.1fs]" % (prelude, out["ms_per_step"], out["value"], wall * 1e3, host[10] * 1e3,
                                    host[-1] * 1e3, time.time() - t0), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
