#!/usr/bin/env python3
"""Time the pair-batch path (hbtc_verify_ciphertexts, RLC and per-share) on N valid ciphertexts:
a kernel-level probe for rocprofv3 (usage: tools/pb_probe.py [N] [reps])."""
import os
import random
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from hbbft_amd import _native as N  # noqa: E402

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
G1 = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
G2 = bytes.fromhex("93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
                   "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    rng = random.Random(1)
    ctx = N.Context(0)
    d = 256
    rs = [rng.randrange(1, R) for _ in range(d)]
    hs = [rng.randrange(1, R) for _ in range(d)]
    u = np.frombuffer(bytes(ctx.g1_mul(G1, rs)[0]), np.uint8).reshape(d, 48)
    H = np.frombuffer(bytes(ctx.g2_mul(G2, hs)[0]), np.uint8).reshape(d, 96)
    w = np.frombuffer(bytes(ctx.g2_mul(G2, [r * h % R for r, h in zip(rs, hs)])[0]), np.uint8).reshape(d, 96)
    pick = np.array([rng.randrange(d) for _ in range(n)])
    us, Hs, ws = u[pick].copy(), H[pick].copy(), w[pick].copy()
    ctx.timing_enable(True)
    for mode, name in ((N.MODE_RLC, "rlc"), (N.MODE_PER_SHARE, "per_share")):
        ctx.set_verify_mode(mode)
        ctx.verify_ciphertexts(us, Hs, ws)
        ctx.timing_reset()
        t0 = time.perf_counter()
        for _ in range(reps):
            st = ctx.verify_ciphertexts(us, Hs, ws)
        dt = (time.perf_counter() - t0) / reps
        assert (st == N.ACCEPT).all()
        spans = {f: round(ctx.timing_read(f)[0] / reps, 3) for f in
                 ("pb_items", "pb_lines", "pb_ml", "pb_checks", "pair_verify") if ctx.timing_read(f)[1]}
        print("%s: %d ciphertexts in %.1f ms (%.0f /s); spans ms %s" % (name, n, dt * 1e3, n / dt, spans),
              flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
