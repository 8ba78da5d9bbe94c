"""CPU baseline leg of bench.py (TEST / BASELINE INFRASTRUCTURE ONLY): the Python restatement of
threshold_crypto's per-call DecryptionShare check, timed on a bounded sample of the benchmark's
own workload across a process pool on this host's cores.

Per share this is exactly what hbbft pays per received share (src/threshold_decryption.rs:152-161
-> PublicKeyShare::verify_decryption_share): serde decode of the share (on-curve + r-torsion
check, pairing 0.14 into_affine), hash_g1_g2(u, v) recomputed on every call, and two full
pairings compared.  Used only when the C restatement (oracle/cbaseline.py) is not built.
"""
import multiprocessing as mp
import os
import random
import time

from . import bls12_381 as B
from . import threshold_crypto as T


def _worker(args):
    shares, pk, u, v, w, budget = args
    t0 = time.perf_counter()
    done = 0
    ok = 0
    for enc in shares:
        d = B.g1_decompress(enc)
        H = T.hash_g1_g2(u, v)
        ok += T.verify_decryption_share_h(pk, d, H, w)
        done += 1
        if time.perf_counter() - t0 > budget:
            break
    return done, ok, time.perf_counter() - t0


def run_dec_share_baseline(ep, budget_s, cores=None):
    cores = cores or min(16, os.cpu_count() or 1)
    rng = random.Random(1)
    # one ciphertext of the workload (k = 0): u = r G1, w = r H; shares of node 0..n-1
    r = ep.rs[0]
    u = B.g1_mul(B.G1_GEN, r)
    v = bytes(rng.randrange(256) for _ in range(64))
    w = B.g2_mul(B.g2_mul(B.G2_GEN, rng.randrange(1, B.R)), r)  # structure only; timing is data-independent
    pk = B.g1_decompress(bytes(ep.host_shares[0]))  # any valid G1 point
    per = max(1, 64 // cores)
    jobs = []
    for c in range(cores):
        sl = [bytes(ep.host_shares[(c * per + j) % ep.n]) for j in range(per * 4)]
        jobs.append((sl, pk, u, v, w, budget_s))
    t0 = time.perf_counter()
    with mp.get_context("spawn").Pool(cores) as pool:
        res = pool.map(_worker, jobs)
    wall = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    return {
        "value": round(done / wall, 3),
        "unit": "shares/s",
        "cores": cores,
        "kind": "port",
        "impl": "python oracle (oracle/threshold_crypto.py)",
        "sample": "%d DecryptionShare checks of ciphertext 0 (serde decode + hash_g1_g2 + 2 pairings each), "
                  "%d processes, %.1fs wall" % (done, cores, wall),
    }
