"""GPU parity of the batched Pippenger MSM (hbtc_g1_msm / hbtc_g2_msm) and of the combines built
on it, including "combine from the verified shares" (hbtc_combine_*_verified_dev).

Oracle: small MSMs against the Python restatement (oracle/bls12_381.py: sum of independent
double-and-add multiplications, as threshold_crypto's interpolate / Commitment::evaluate do);
larger ones through the size-independent identity sum_i k_i (a_i G) == (sum_i k_i a_i) G.
Bar: byte-identical compressed points (integer arithmetic, no tolerance).
"""
import ctypes
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from oracle import bls12_381 as B
from oracle import threshold_crypto as TC

pytestmark = pytest.mark.gpu

R = B.R
G1 = B.g1_compress(B.G1_GEN)
G2 = B.g2_compress(B.G2_GEN)


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    yield c
    c.close()


def _pts(ctx, group, scal):
    if group == 1:
        out, st = ctx.g1_mul(G1, scal)
        size = 48
    else:
        out, st = ctx.g2_mul(G2, scal)
        size = 96
    assert not st.any()
    return [bytes(out[size * i:size * i + size]) for i in range(len(scal))]


def _gen(ctx, group, vals):
    """[v] G compressed, via the library (checked against the oracle in test_gpu_parity)."""
    return _pts(ctx, group, [v % R for v in vals])


@pytest.mark.parametrize("group", [1, 2])
def test_msm_small_vs_oracle(ctx, group):
    rng = random.Random(11 + group)
    n_msm, n = 3, 6
    a = [rng.randrange(1, R) for _ in range(n_msm * n)]
    k = [rng.randrange(0, R) for _ in range(n_msm * n)]
    pts = _gen(ctx, group, a)
    msm = ctx.g1_msm if group == 1 else ctx.g2_msm
    out, st = msm(n_msm, n, pts, k)
    assert not st.any()
    dec = B.g1_decompress if group == 1 else B.g2_decompress
    mul = B.g1_mul if group == 1 else B.g2_mul
    add = B.g1_add if group == 1 else B.g2_add
    comp = B.g1_compress if group == 1 else B.g2_compress
    for m in range(n_msm):
        acc = None
        for i in range(n):
            term = mul(dec(pts[m * n + i]), k[m * n + i])
            acc = term if acc is None else add(acc, term)
        assert out[m] == comp(acc)


@pytest.mark.parametrize("group,n", [(1, 1), (1, 7), (1, 64), (1, 334), (1, 3000), (2, 34),
                                     (2, 700), (1, 56000), (2, 4000)])
def test_msm_identity(ctx, group, n):
    """sum_i k_i (a_i G) == (sum_i k_i a_i) G across window widths c = 4 .. 12 (n = 56000 is a
    SyncKeyGen Part's MSM at t = 333)."""
    rng = random.Random(1000 * group + n)
    n_msm = 4
    a = [rng.randrange(1, R) for _ in range(n_msm * n)]
    k = [rng.randrange(0, R) for _ in range(n_msm * n)]
    pts = _gen(ctx, group, a)
    msm = ctx.g1_msm if group == 1 else ctx.g2_msm
    out, st = msm(n_msm, n, pts, k)
    assert not st.any()
    want = _gen(ctx, group, [sum(k[m * n + i] * a[m * n + i] for i in range(n)) % R
                             for m in range(n_msm)])
    assert out == want


@pytest.mark.parametrize("group,n", [(1, 5000), (2, 1500)])
def test_msm_crowded_buckets(ctx, group, n):
    """Scalars K + i share every digit above the lowest windows, so each of those windows puts
    all n terms into ONE bucket: the bucket pass must split that bucket's run over lanes (equal
    slices of the sorted list) and still sum to sum_b b B_b."""
    rng = random.Random(77 + group)
    n_msm = 2
    K = rng.randrange(R // 2, R - n)
    a = [rng.randrange(1, R) for _ in range(n_msm * n)]
    k = [K + (i % n) for i in range(n_msm * n)]
    pts = _gen(ctx, group, a)
    msm = ctx.g1_msm if group == 1 else ctx.g2_msm
    out, st = msm(n_msm, n, pts, k)
    assert not st.any()
    want = _gen(ctx, group, [sum(k[m * n + i] * a[m * n + i] for i in range(n)) % R
                             for m in range(n_msm)])
    assert out == want


@pytest.mark.parametrize("group", [1, 2])
def test_msm_edge_scalars_and_points(ctx, group):
    """Scalars 0, 1, r-1, r, 2^256-1; repeated points (bucket doubling), P and -P (cancel to
    infinity inside a bucket), the identity point, and an invalid encoding -> DECODE_ERR."""
    rng = random.Random(77 + group)
    size = 48 if group == 1 else 96
    msm = ctx.g1_msm if group == 1 else ctx.g2_msm
    a = [rng.randrange(1, R) for _ in range(4)]
    base = _gen(ctx, group, a)
    neg0 = _gen(ctx, group, [R - a[0]])[0]
    inf = bytes([0xC0]) + bytes(size - 1)
    pts = [base[0], base[0], base[1], neg0, inf, base[2], base[3], base[0]]
    ks = [5, 5, 0, 5, 12345, R - 1, R, (1 << 256) - 1]
    av = [a[0], a[0], a[1], R - a[0], 0, a[2], a[3], a[0]]
    out, st = msm(1, len(pts), pts, ks)
    assert list(st) == [N.ACCEPT]
    want = _gen(ctx, group, [sum(k * v for k, v in zip(ks, av)) % R])
    if sum(k * v for k, v in zip(ks, av)) % R == 0:
        want = [inf]
    assert out == want
    # all terms cancel: infinity
    out, st = msm(1, 2, [base[0], neg0], [9, 9])
    assert list(st) == [N.ACCEPT] and out == [inf]
    # invalid encoding (compression flag cleared)
    bad = bytearray(base[1])
    bad[0] &= 0x7F
    out, st = msm(2, 2, [base[0], base[1], bytes(bad), base[2]], [1, 2, 3, 4])
    assert list(st) == [N.ACCEPT, N.DECODE_ERR]


def _dev(ctx, arr):
    a = np.ascontiguousarray(arr)
    p = ctx.dev_alloc(max(a.nbytes, 16))
    if a.nbytes:
        ctx.dev_upload(p, a)
    return p


@pytest.mark.parametrize("mode", [N.MODE_RLC, N.MODE_PER_SHARE])
def test_decrypt_combine_from_verified_shares(ctx, mode):
    """ThresholdDecryption semantics (td.rs:184): the combine uses the first t VERIFIED shares.
    Wrong shares among the first t are skipped; too few verified shares -> NOT_ENOUGH_SHARES."""
    rng = random.Random(5)
    n, t, n_ct = 16, 6, 4
    coeffs = [rng.randrange(1, R) for _ in range(t)]
    sks = [sum(c * pow(i + 1, j, R) for j, c in enumerate(coeffs)) % R for i in range(n)]
    pk = _gen(ctx, 1, sks)
    ks, nbad = ctx.keyset_load(pk)
    assert nbad == 0
    rs = [rng.randrange(1, R) for _ in range(n_ct)]
    hs = [rng.randrange(1, R) for _ in range(n_ct)]
    H = _gen(ctx, 2, hs)
    w = _gen(ctx, 2, [r * h for r, h in zip(rs, hs)])
    wrong = {0: {0, 2}, 1: set(), 2: set(range(0, n - t + 1)), 3: {5}}  # ct 2: only t-1 good
    scal = []
    for k in range(n_ct):
        for i in range(n):
            s = sks[i] * rs[k] % R
            scal.append((s + 1) % R if i in wrong[k] else s)
    shares = np.frombuffer(b"".join(_gen(ctx, 1, scal)), np.uint8).copy()
    idx = np.tile(np.arange(n, dtype=np.uint32), n_ct)
    off = np.arange(0, n * n_ct + 1, n, dtype=np.uint32)
    ctx.set_verify_mode(mode)
    try:
        d_H = _dev(ctx, np.frombuffer(b"".join(H), np.uint8))
        d_w = _dev(ctx, np.frombuffer(b"".join(w), np.uint8))
        d_idx, d_sh = _dev(ctx, idx), _dev(ctx, shares)
        d_st = ctx.dev_alloc(4 * n * n_ct)
        d_g, d_cst = ctx.dev_alloc(48 * n_ct), ctx.dev_alloc(4 * n_ct)
        lib, h = ctx.lib, ctx.h
        offp = N._ptr(off)
        ctx._check(lib.hbtc_verify_dec_shares_dev(h, ks, n_ct, d_H, d_w, offp, d_idx, d_sh, d_st),
                   "verify")
        ctx._check(lib.hbtc_combine_dec_verified_dev(h, n_ct, offp, d_idx, d_sh, d_st, t, d_g,
                                                     d_cst), "combine verified")
        st = np.empty(n * n_ct, np.int32)
        ctx.dev_download(st, d_st)
        g = np.empty(48 * n_ct, np.uint8)
        ctx.dev_download(g, d_g)
        cst = np.empty(n_ct, np.int32)
        ctx.dev_download(cst, d_cst)
    finally:
        ctx.set_verify_mode(N.MODE_RLC)
    exp = [N.REJECT if i in wrong[k] else N.ACCEPT for k in range(n_ct) for i in range(n)]
    assert list(st) == exp
    assert list(cst) == [N.ACCEPT, N.ACCEPT, N.NOT_ENOUGH_SHARES, N.ACCEPT]
    want = _gen(ctx, 1, [coeffs[0] * r for r in rs])
    for k in (0, 1, 3):
        assert bytes(g[48 * k:48 * k + 48]) == want[k]
    assert bytes(g[96:144]) == bytes(48)


def test_sig_combine_from_verified_shares(ctx):
    """Coin semantics (coin.rs:185-191): combine the first t verified signature shares; the
    parity bit equals the one of master_sk * H."""
    rng = random.Random(9)
    n, t, n_inst = 10, 4, 3
    coeffs = [rng.randrange(1, R) for _ in range(t)]
    sks = [sum(c * pow(i + 1, j, R) for j, c in enumerate(coeffs)) % R for i in range(n)]
    ks, _ = ctx.keyset_load(_gen(ctx, 1, sks))
    hs = [rng.randrange(1, R) for _ in range(n_inst)]
    H = _gen(ctx, 2, hs)
    wrong = {0: {1}, 1: {0, 1, 2}, 2: set()}
    scal = [(sks[i] * hs[k] + (1 if i in wrong[k] else 0)) % R
            for k in range(n_inst) for i in range(n)]
    sigs = np.frombuffer(b"".join(_gen(ctx, 2, scal)), np.uint8).copy()
    idx = np.tile(np.arange(n, dtype=np.uint32), n_inst)
    off = np.arange(0, n * n_inst + 1, n, dtype=np.uint32)
    d_H = _dev(ctx, np.frombuffer(b"".join(H), np.uint8))
    d_idx, d_sig = _dev(ctx, idx), _dev(ctx, sigs)
    d_st = ctx.dev_alloc(4 * n * n_inst)
    d_out, d_par, d_cst = ctx.dev_alloc(96 * n_inst), ctx.dev_alloc(16), ctx.dev_alloc(4 * n_inst)
    lib, h = ctx.lib, ctx.h
    offp = N._ptr(off)
    ctx._check(lib.hbtc_verify_sig_shares_dev(h, ks, n_inst, d_H, offp, d_idx, d_sig, d_st), "v")
    ctx._check(lib.hbtc_combine_sigs_verified_dev(h, n_inst, offp, d_idx, d_sig, d_st, t, d_out,
                                                  d_par, d_cst), "c")
    out = np.empty(96 * n_inst, np.uint8)
    ctx.dev_download(out, d_out)
    par = np.empty(16, np.uint8)
    ctx.dev_download(par, d_par)
    cst = np.empty(n_inst, np.int32)
    ctx.dev_download(cst, d_cst)
    assert list(cst) == [N.ACCEPT] * n_inst
    want = _gen(ctx, 2, [coeffs[0] * hv for hv in hs])
    for k in range(n_inst):
        got = bytes(out[96 * k:96 * k + 96])
        assert got == want[k]
        # Signature::parity restated by the oracle (XOR-popcount of the uncompressed encoding)
        assert bool(par[k]) == TC.signature_parity(B.g2_decompress(got))
