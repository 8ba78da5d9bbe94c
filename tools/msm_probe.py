#!/usr/bin/env python3
"""Probe: G1 Pippenger bucket-reduction rate (mixed adds / s) against MSM size and batch size,
through hbtc_g1_msm.  Usage: python tools/msm_probe.py  (GPU)."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hbbft_amd import _native as N  # noqa: E402

G1_GEN = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")


def main():
    ctx = N.Context(0)
    rng = np.random.default_rng(1)
    base_n = 56000
    sc = rng.integers(0, 256, size=(base_n, 32), dtype=np.uint8)
    sc[:, 31] &= 0x3F
    pts, st = ctx.g1_mul(G1_GEN, sc.reshape(-1))
    assert not st.any()
    pts = pts.reshape(base_n, 48)
    ctx.timing_enable(True)
    for n, n_msm in ((335, 1000), (4096, 64), (56000, 4), (56000, 16), (56000, 64)):
        P = np.ascontiguousarray(np.tile(pts[:n], (n_msm, 1)))
        S = rng.integers(0, 256, size=(n_msm * n, 32), dtype=np.uint8)
        S[:, 31] &= 0x3F
        ctx.g1_msm(n_msm, n, P, S)  # warm
        ctx.timing_reset()
        t0 = time.perf_counter()
        ctx.g1_msm(n_msm, n, P, S)
        dt = time.perf_counter() - t0
        comb, k = ctx.timing_read("combine")
        dec, _ = ctx.timing_read("comb_decode")
        print("n=%6d n_msm=%5d terms=%9d wall %.1f ms, decode %.1f ms, reduce %.1f ms (%d launches), "
              "reduce ns/term %.2f" % (n, n_msm, n * n_msm, dt * 1e3, dec, comb, k,
                                       comb * 1e6 / (n * n_msm)), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
