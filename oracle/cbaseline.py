"""ctypes binding of the C restatement oracle/c/libtcoracle.so — TEST / BASELINE ONLY.

Used by tests/ (cross-checks against the Python oracle and the golden fixtures) and by
bench.py's cpu_baseline leg (the reference's per-call algorithm over a pthread pool on the
host's cores).  Raises ImportError when the library is not built, so bench.py can fall back to
the Python restatement for the baseline.
"""
import ctypes
import os
import random
import time

_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "c", "libtcoracle.so")
if not os.path.exists(_PATH):
    raise ImportError("oracle/c/libtcoracle.so not built (make oracle)")
_lib = ctypes.CDLL(_PATH)
_B = ctypes.c_char_p
_lib.tco_init.restype = None
_lib.tco_pairing_eq.argtypes = [_B, _B, _B, _B]
_lib.tco_g1_mul.argtypes = [_B, _B, ctypes.c_void_p]
_lib.tco_g2_mul.argtypes = [_B, _B, ctypes.c_void_p]
_lib.tco_hash_g2.argtypes = [_B, ctypes.c_size_t, ctypes.c_void_p]
_lib.tco_hash_g2.restype = None
_lib.tco_hash_g1_g2.argtypes = [_B, _B, ctypes.c_size_t, ctypes.c_void_p]
_lib.tco_hash_g1_g2.restype = None
_lib.tco_sha3_256.argtypes = [_B, ctypes.c_size_t, ctypes.c_void_p]
_lib.tco_sha3_256.restype = None
_lib.tco_sig_parity.argtypes = [_B]
_lib.tco_combine_g1.argtypes = [ctypes.c_uint32, ctypes.c_void_p, _B, ctypes.c_uint32, ctypes.c_void_p]
_lib.tco_combine_g2.argtypes = [ctypes.c_uint32, ctypes.c_void_p, _B, ctypes.c_uint32, ctypes.c_void_p]
_lib.tco_bench_dec_shares.restype = ctypes.c_uint64
_lib.tco_bench_dec_shares.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_double, _B, ctypes.c_uint32,
                                      _B, _B, _B, ctypes.c_size_t, _B,
                                      ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]
_lib.tco_bench_sig_shares.restype = ctypes.c_uint64
_lib.tco_bench_sig_shares.argtypes = [ctypes.c_int, ctypes.c_double, _B, _B, ctypes.c_uint32, _B,
                                      ctypes.c_size_t, ctypes.POINTER(ctypes.c_double),
                                      ctypes.POINTER(ctypes.c_uint64)]
_lib.tco_bench_g1_mul.restype = ctypes.c_uint64
_lib.tco_bench_g1_mul.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.POINTER(ctypes.c_double)]
_lib.tco_init()


def pairing_eq(p1, q1, p2, q2):
    """e(p1, q1) == e(p2, q2) by two full pairings: True/False, None on a decode error."""
    r = _lib.tco_pairing_eq(bytes(p1), bytes(q1), bytes(p2), bytes(q2))
    return None if r < 0 else bool(r)


def g1_mul(p48, k):
    out = ctypes.create_string_buffer(48)
    if _lib.tco_g1_mul(bytes(p48), int(k).to_bytes(32, "little"), out) != 0:
        return None
    return out.raw


def g2_mul(p96, k):
    out = ctypes.create_string_buffer(96)
    if _lib.tco_g2_mul(bytes(p96), int(k).to_bytes(32, "little"), out) != 0:
        return None
    return out.raw


def sha3_256(msg):
    out = ctypes.create_string_buffer(32)
    _lib.tco_sha3_256(bytes(msg), len(msg), out)
    return out.raw


def hash_g2(msg):
    out = ctypes.create_string_buffer(96)
    _lib.tco_hash_g2(bytes(msg), len(msg), out)
    return out.raw


def hash_g1_g2(g1_48, msg):
    out = ctypes.create_string_buffer(96)
    _lib.tco_hash_g1_g2(bytes(g1_48), bytes(msg), len(msg), out)
    return out.raw


def sig_parity(sig96):
    return _lib.tco_sig_parity(bytes(sig96))


def combine(group, idx, pts, t):
    """(status, bytes): status 0 ok, 5 NotEnoughShares, 6 DuplicateEntry, 2 decode error."""
    size = 48 if group == 1 else 96
    n = len(idx)
    ix = (ctypes.c_uint32 * max(n, 1))(*idx)
    out = ctypes.create_string_buffer(size)
    fn = _lib.tco_combine_g1 if group == 1 else _lib.tco_combine_g2
    st = fn(n, ix, b"".join(bytes(p) for p in pts), t, out)
    return st, (out.raw if st == 0 else None)


def bench_dec_shares(mode, threads, budget_s, shares, pk48, u48, v, w96):
    """Run the C baseline: mode 0 = threshold_crypto's per-call path, 1 = optimized CPU."""
    wall, acc = ctypes.c_double(), ctypes.c_uint64()
    blob = b"".join(bytes(s) for s in shares)
    done = _lib.tco_bench_dec_shares(mode, threads, budget_s, blob, len(shares), bytes(pk48),
                                     bytes(u48), bytes(v), len(v), bytes(w96), ctypes.byref(wall),
                                     ctypes.byref(acc))
    return int(done), wall.value, int(acc.value)


def host_cpus():
    """The host's CPUs as this process may use them: nproc (os.cpu_count), the affinity mask,
    the cgroup CPU quota (cpu.max) and the CPU model.  `usable` = min(affinity, quota): every
    core the scheduler will actually give the baseline's threads (on a shared GPU box the quota
    is the box's CPU share, e.g. 16 of a 192-CPU machine)."""
    nproc = os.cpu_count() or 1
    try:
        aff = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        aff = nproc
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) // int(per)))
        except (OSError, ValueError):
            pass
    if quota is None:
        try:
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0:
                quota = max(1, q // per)
        except (OSError, ValueError):
            pass
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    usable = min(aff, quota) if quota else aff
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit() and quota is None and usable > int(env) > 0:
        usable = int(env)  # the box's stated CPU share when no cgroup quota is visible
    return {"nproc": nproc, "affinity": aff, "cgroup_quota": quota, "model": model, "usable": usable}


def run_dec_share_baseline(ep, budget_s, cores=None):
    """bench.py cpu_baseline leg: the reference-faithful per-call path on every core this process
    may use (host_cpus()['usable']), on real decryption shares of the benchmark's ciphertext 0."""
    cpus = host_cpus()
    cores = cores or cpus["usable"]
    rng = random.Random(3)
    k = 0
    shares = [bytes(ep.host_shares[k * ep.n + i]) for i in range(ep.n)]
    # ciphertext 0's own u / w / pk_0 in compressed form
    pk0 = ep.pk_bytes[0]
    u = ep.u_bytes[k]
    w = ep.w_bytes[k]
    v = bytes(rng.randrange(256) for _ in range(64))
    done, wall, acc = bench_dec_shares(0, cores, budget_s, shares, pk0, u, v, w)
    done_o, wall_o, _ = bench_dec_shares(1, cores, min(10.0, budget_s / 2), shares, pk0, u, v, w)
    return {
        "value": round(done / wall, 2),
        "unit": "shares/s",
        "cores": cores,
        "host_cpus": cpus,
        "kind": "port",
        "impl": "C restatement of threshold_crypto 0.1 / pairing 0.14 (oracle/c/tc_oracle.c), pthreads",
        "sample": "%d DecryptionShare checks of ciphertext 0 in %.1fs: per share serde decode ([r]P "
                  "subgroup check) + hash_g1_g2(u, v) + two full pairings, as hbbft calls "
                  "verify_decryption_share (src/threshold_decryption.rs:159)" % (done, wall),
        "optimized_cpu": {"value": round(done_o / wall_o, 2), "unit": "shares/s",
                          "sample": "%d shares in %.1fs: hash + G2 preparation once per ciphertext, one "
                                    "2-pair multi-Miller loop + one final exponentiation per share"
                                    % (done_o, wall_o)},
    }


def run_sig_share_baseline(sigs96, pks48, nonce, budget_s, cores=None):
    """bench_configs.py c2 / c4 cpu_baseline: the reference-faithful PublicKeyShare::verify
    (src/coin.rs:151: serde decode of the share, hash_g2(nonce) per call, two full pairings) on
    every usable core, over real shares of the benchmark's first instance (share i with its
    sender's pk)."""
    cpus = host_cpus()
    cores = cores or cpus["usable"]
    n = len(pks48) // 48
    wall, acc = ctypes.c_double(), ctypes.c_uint64()
    done = _lib.tco_bench_sig_shares(cores, budget_s, bytes(sigs96), bytes(pks48), n, bytes(nonce), len(nonce),
                                     ctypes.byref(wall), ctypes.byref(acc))
    return {"value": round(done / wall.value, 2), "unit": "shares/s", "cores": cores, "host_cpus": cpus,
            "kind": "port",
            "impl": "C restatement of threshold_crypto 0.1 / pairing 0.14 (oracle/c/tc_oracle.c), pthreads",
            "sample": "%d SignatureShare checks of instance 0 in %.1fs: per share serde decode ([r]Q subgroup "
                      "check) + hash_g2(nonce) + two full pairings, as Coin calls PublicKeyShare::verify "
                      "(src/coin.rs:151)" % (done, wall.value)}


def run_skg_ack_baseline(n, t, budget_s, cores=None):
    """bench_configs.py c5 cpu_baseline: the reference's Ack check is
    commit.evaluate(x, y) == val * G1 (src/sync_key_gen.rs:493), i.e. (t+1)^2 G1 scalar
    multiplications per Ack (BivarCommitment::evaluate over the (t+1)^2 coefficient grid) plus
    the Ack value's SecretKey::decrypt (two pairings, :483).  At N = 1000 one Ack is ~112k
    scalar multiplications, so the sample times the scalar multiplication on every usable core
    and reports the Acks/s that rate gives (the decrypt's pairings are left out: a lower bound on
    the reference's time, an upper bound on its rate)."""
    cpus = host_cpus()
    cores = cores or cpus["usable"]
    wall = ctypes.c_double()
    done = _lib.tco_bench_g1_mul(cores, budget_s, ctypes.byref(wall))
    per_ack = (t + 1) ** 2
    rate = done / wall.value
    return {"value": round(rate / per_ack, 4), "unit": "acks/s (projected from the timed scalar multiplications)",
            "cores": cores, "host_cpus": cpus, "kind": "port",
            "impl": "C restatement of pairing 0.14's G1 double-and-add (oracle/c/tc_oracle.c), pthreads",
            "sample": "%d G1 scalar multiplications in %.1fs (%.0f /s); one Ack = (t+1)^2 = %d of them "
                      "(commit.evaluate at N = %d, t = %d), decrypt pairings excluded"
                      % (done, wall.value, rate, per_ack, n, t)}


def _median(xs):
    s = sorted(xs)
    return s[len(s) // 2]


def coin_call(sigs96, pks48, master_pk48, nonce, t, pool=None):
    """One Coin call as hbbft makes it (src/coin.rs:149-207), by the C restatement: every
    SignatureShare through PublicKeyShare::verify (serde decode with the subgroup check,
    hash_g2(nonce) inside each call, two full pairings; coin.rs:151), the first t valid ones
    through combine_signatures (Lagrange in G2, :185-191), the result through PublicKey::verify
    against the master key (:192-197) and Signature::parity (:173).  pool: a thread pool for the
    share checks (ctypes drops the GIL inside the C calls), None = one core.
    Returns (statuses, combined signature, parity)."""
    n = len(pks48) // 48
    g1 = bytes.fromhex("97f1d3a73197d7942695638c4fa9ac0fc3688c4f9774b905a14e3a3f171bac58"
                       "6c55e83ff97a1aeffb3af00adb22c6bb")

    def check(i):
        H = hash_g2(nonce)
        return pairing_eq(pks48[48 * i:48 * i + 48], H, g1, sigs96[96 * i:96 * i + 96])

    ok = list(pool.map(check, range(n))) if pool else [check(i) for i in range(n)]
    sel = [i for i in range(n) if ok[i]][:t]
    st, sig = combine(2, sel, [sigs96[96 * i:96 * i + 96] for i in sel], t)
    if st != 0:
        return ok, None, None
    H = hash_g2(nonce)
    assert pairing_eq(master_pk48, H, g1, sig)
    return ok, sig, sig_parity(sig)


def run_coin_call_baseline(sigs96, pks48, master_pk48, nonce, t, budget_s=10.0):
    """Single-call latency of coin_call on one core and on every usable core (a thread pool over
    the share checks), each repeated for about budget_s / 2."""
    from concurrent.futures import ThreadPoolExecutor
    cpus = host_cpus()
    res = {}
    for cores in (1, cpus["usable"]):
        pool = ThreadPoolExecutor(cores) if cores > 1 else None
        lat = []
        t_end = time.perf_counter() + budget_s / 2
        while True:
            a = time.perf_counter()
            ok, sig, par = coin_call(sigs96, pks48, master_pk48, nonce, t, pool)
            lat.append(time.perf_counter() - a)
            if time.perf_counter() > t_end and len(lat) >= 3:
                break
        if pool:
            pool.shutdown()
        res[cores] = (lat, ok, sig, par)
    one, many = res[1], res[cpus["usable"]]
    return {"value": round(1e3 * _median(one[0]), 3), "unit": "ms per coin call (median, 1 core)",
            "value_all_cores_ms": round(1e3 * _median(many[0]), 3), "cores": 1,
            "cores_all": cpus["usable"], "host_cpus": cpus, "kind": "port",
            "calls": [len(one[0]), len(many[0])], "results": (one[1], one[2], one[3]),
            "impl": "C restatement of threshold_crypto 0.1 / pairing 0.14 (oracle/c/tc_oracle.c) driven "
                    "per call; the share checks over a thread pool for the all-cores figure",
            "sample": "repeated whole coin calls (%d shares: decode + hash_g2 + 2 pairings each; combine of "
                      "t = %d; master PublicKey::verify; parity)" % (len(pks48) // 48, t)}
