"""Debug: the coin_decide test's 64-instance case (RLC path) on fresh / reused contexts."""
import json, os, random, sys
sys.path.insert(0, os.getcwd())
import numpy as np
from hbbft_amd import _native as N
from oracle import bls12_381 as B
sys.path.insert(0, "tests")
import test_gpu_coin_decide as T

R = B.R
def case(n=10, t=4, n_inst=64):
    rng = random.Random(31 * n + t + n_inst)
    poly = [rng.randrange(1, R) for _ in range(t)]
    sks = [sum(c * pow(i + 1, e, R) for e, c in enumerate(poly)) % R for i in range(n)]
    ctx = N.Context(0)
    g1 = B.g1_compress(B.G1_GEN); g2 = B.g2_compress(B.G2_GEN)
    pk, st = ctx.g1_mul(g1, sks)
    mpk, _ = ctx.g1_mul(g1, [poly[0]])
    wrong_mpk, _ = ctx.g1_mul(g1, [(poly[0] + 1) % R])
    hs = [rng.randrange(1, R) for _ in range(n_inst)]
    Hs, _ = ctx.g2_mul(g2, hs)
    H = [bytes(Hs[96 * k:96 * k + 96]) for k in range(n_inst)]
    codec = json.load(open("tests/golden/codec.json"))
    bad2 = [bytes.fromhex(x["enc"]) for x in codec["g2_bad"]]
    counts, idx, scal, edits, kinds = T._instances(rng, n, t, n_inst, sks, hs, bad2)
    sg, st2 = ctx.g2_mul(g2, scal)
    sigs = [bytes(sg[96 * i:96 * i + 96]) for i in range(len(scal))]
    for pos, enc in edits:
        sigs[pos] = enc
    ctx.close()
    return pk, counts, idx, sigs, H, kinds

pk, counts, idx, sigs, H, kinds = case()
def run(label, warm_small=False):
    c = N.Context(0)
    ks, _ = c.keyset_load(pk)
    if warm_small:
        c.verify_sig_shares(ks, H[:8], counts[:8], idx[:sum(counts[:8])], sigs[:sum(counts[:8])])
    a = c.verify_sig_shares(ks, H, counts, idx, sigs)
    b = c.verify_sig_shares(ks, H, counts, idx, sigs)
    c.close()
    return a, b
res = {}
for label, warm in (("fresh", False), ("after_small", True)):
    a, b = run(label, warm)
    res[label] = a
    print(label, "first/second equal:", bool((a == b).all()), "accepts", int((a == 0).sum()), int((b == 0).sum()), flush=True)
print("fresh vs after_small equal:", bool((res["fresh"] == res["after_small"]).all()))
d = np.nonzero(res["fresh"] != res["after_small"])[0]
print("diff positions", d[:20], res["fresh"][d[:20]], res["after_small"][d[:20]])
# expected from the kinds: valid instance shares ACCEPT
pos = 0
bad = []
for k, (cnt, kind) in enumerate(zip(counts, kinds)):
    if kind == "valid":
        for j in range(pos, pos + cnt):
            if res["fresh"][j] != 0 or res["after_small"][j] != 0:
                bad.append((k, j, int(res["fresh"][j]), int(res["after_small"][j])))
    pos += cnt
print("valid-instance non-accepts (inst, item, fresh, after_small):", bad[:20], len(bad))
