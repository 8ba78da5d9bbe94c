"""Step-by-step GPU sanity run with a progress line per step (debug tool)."""
import sys, time
sys.path.insert(0, ".")
from hbbft_amd import _native as N
def log(*a):
    print(*a, flush=True)
t0 = time.time()
ctx = N.Context(0)
log("ctx", round(time.time() - t0, 2))
G1 = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac586c55e83ff97a1aeffb3af00adb22c6bb")
for n in (1, 64, 4096):
    t0 = time.time()
    out, st = ctx.g1_mul(G1, list(range(1, n + 1)))
    log("g1_mul", n, round(time.time() - t0, 3), st[:4])
G2 = bytes.fromhex("93e02b6052719f607dacd3a088274f65596bd0d09920b61ab5da61bbdc7f5049334cf11213945d57e5ac7d055d042b7e"
                   "024aa2b2f08f0a91260805272dc51051c6e47ad4fa403b02b4510b647ae3d1770bac0326a805bbefd48056c8c121bdb8")
for n in (1, 64):
    t0 = time.time()
    out, st = ctx.g2_mul(G2, list(range(1, n + 1)))
    log("g2_mul", n, round(time.time() - t0, 3), st[:4])
t0 = time.time()
bad = bytearray(G1); bad[0] &= 0x7F
_, st = ctx.g1_mul([bytes(bad)], [1])
log("g1 bad", round(time.time() - t0, 3), st)
t0 = time.time()
pk, _ = ctx.g1_mul(G1, list(range(1, 11)))
ks, nb = ctx.keyset_load(pk)
log("keyset", round(time.time() - t0, 3), nb)
