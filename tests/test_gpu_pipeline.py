"""Pipelined host-buffer epochs (hbtc_dec_epoch_submit / hbtc_sig_epoch_submit / hbtc_wait,
include/hbtc.h): several epochs in flight give exactly the results of the blocking calls
(hbtc_verify_*_shares + the combine of the first t ACCEPTed shares of every instance), with a
fifth submit completing the oldest, out-of-order waits, t = 0 (verification only), empty
batches and inputs overwritten right after submit (the library copies them)."""
import random

import numpy as np
import pytest

from hbbft_amd import _native as N
from tests.test_gpu_parity import _dec_batch, _sig_batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    c.set_verify_mode(N.MODE_RLC)
    c.set_exact_below(0)
    yield c
    c.close()


def _first_t_verified(st, off, t):
    """The blocking reference: the first t ACCEPTed items of every instance (positions)."""
    sel = []
    for k in range(len(off) - 1):
        acc = [i for i in range(off[k], off[k + 1]) if st[i] == N.ACCEPT]
        sel.append(acc[:t])
    return sel


def test_dec_epochs_in_flight_equal_blocking_calls(ctx):
    rng = random.Random(71)
    n = 40
    t = (n - 1) // 3 + 1
    batches = []
    for e in range(7):
        counts = [40, 0, 7, 64, 65, 1, 130, 33][: 3 + e % 6]
        pk, H, w, idx, shares, _, _ = _dec_batch(ctx, rng, n, counts, 0.05 * (e % 3))
        ks, _ = ctx.keyset_load(pk)
        off = np.zeros(len(counts) + 1, np.uint32)
        off[1:] = np.cumsum(counts)
        batches.append((ks, H, w, off, np.asarray(idx, np.uint32), np.asarray(shares, np.uint8).copy()))
    # the blocking reference of every epoch
    want = []
    for ks, H, w, off, idx, sh in batches:
        st = ctx.verify_dec_shares(ks, H, w, None, idx, sh, offsets=off)
        sel = _first_t_verified(st, off, t)
        counts = [len(s) for s in sel]
        flat = [i for s in sel for i in s]
        g, cst = ctx.combine_dec(counts, idx[flat], sh.reshape(-1, 48)[flat].reshape(-1), t)
        want.append((st, g, cst))
    # seven epochs submitted back to back (a fifth submit completes the oldest); inputs are
    # scribbled over after each submit; waits in reverse order
    pend = []
    for ks, H, w, off, idx, sh in batches:
        sh2 = sh.copy()
        pend.append(ctx.dec_epoch_submit(ks, H, w, off, idx, sh2, t))
        sh2[:] = 0
    for e in reversed(range(len(pend))):
        st, g, cst = pend[e].wait()
        wst, wg, wcst = want[e]
        m = len(wcst)
        assert (st[:len(wst)] == wst).all(), e
        assert (cst[:m] == wcst).all(), e
        for k in range(m):
            if wcst[k] == N.ACCEPT:
                assert g[k].tobytes() == wg[k], (e, k)
    # t = 0: verification only; an empty epoch
    ks, H, w, off, idx, sh = batches[0]
    st, _, _ = ctx.dec_epoch_submit(ks, H, w, off, idx, sh, 0).wait()
    assert (st[:len(want[0][0])] == want[0][0]).all()
    p = ctx.dec_epoch_submit(ks, b"", b"", np.zeros(1, np.uint32), np.zeros(0, np.uint32), b"", t)
    p.wait()
    p.wait()  # a completed ticket waits as OK


def test_sig_epochs_in_flight_equal_blocking_calls(ctx):
    rng = random.Random(72)
    n = 40
    t = (n - 1) // 3 + 1
    counts = [40, 0, 7, 64, 65, 1, 130]
    off = np.zeros(len(counts) + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    eps = []
    for e in range(5):
        ks, H, idx, sigs, _, _ = _sig_batch(ctx, rng, n, counts, 0.02 * e)
        eps.append((ks, H, np.asarray(idx, np.uint32), np.asarray(sigs, np.uint8)))
    pend = [ctx.sig_epoch_submit(ks, H, off, idx, sigs, t) for ks, H, idx, sigs in eps]
    for (ks, H, idx, sigs), p in zip(eps, pend):
        st, sig, par, cst = p.wait()
        wst = ctx.verify_sig_shares(ks, H, None, idx, sigs, offsets=off)
        assert (st[:len(wst)] == wst).all()
        sel = _first_t_verified(wst, off, t)
        flat = [i for s in sel for i in s]
        wsig, wpar, wcst = ctx.combine_sigs([len(s) for s in sel], idx[flat],
                                            sigs.reshape(-1, 96)[flat].reshape(-1), t)
        m = len(counts)
        assert (cst[:m] == wcst).all()
        for k in range(m):
            if wcst[k] == N.ACCEPT:
                assert sig[k].tobytes() == wsig[k] and par[k] == wpar[k]


def test_dropped_pending_keeps_outputs_alive(ctx):
    """A Pending dropped without wait(): the Context holds its output arrays, so the unasked
    completion of that ticket by a later submit (lane reuse) writes into live memory, and the
    later epochs still give the blocking calls' results (_native.py:383)."""
    import gc
    rng = random.Random(73)
    n = 40
    t = (n - 1) // 3 + 1
    counts = [40, 7, 64]
    pk, H, w, idx, shares, _, _ = _dec_batch(ctx, rng, n, counts, 0.05)
    ks, _ = ctx.keyset_load(pk)
    off = np.zeros(len(counts) + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    idx = np.asarray(idx, np.uint32)
    sh = np.asarray(shares, np.uint8)
    want = ctx.verify_dec_shares(ks, H, w, None, idx, sh, offsets=off)
    p = ctx.dec_epoch_submit(ks, H, w, off, idx, sh, t)
    held, tk = p.outs[0], p.ticket
    del p
    gc.collect()
    assert len(ctx._inflight) >= 1
    later = [ctx.dec_epoch_submit(ks, H, w, off, idx, sh, t) for _ in range(4)]
    for q in later:
        st, _, _ = q.wait()
        assert (st[:len(want)] == want).all()
    assert ctx.lib.hbtc_wait(ctx.h, tk) == 0  # completed (normally already, by the lane's reuse)
    assert (held[:len(want)] == want).all()
    # the held set stays bounded by MAX_HELD_TICKETS
    for _ in range(N.Context.MAX_HELD_TICKETS + 3):
        ctx.dec_epoch_submit(ks, H, w, off, idx, sh, 0)
    assert len(ctx._inflight) <= N.Context.MAX_HELD_TICKETS
