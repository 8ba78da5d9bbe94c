"""The BASELINE.json configurations at their full sizes through the C ABI (-m gpu), checked
against the construction (every share's decision is known when it is generated; every combine
equals the master key applied to the instance's nonce) and, on slices, against the per-share
mode.  The bench scripts build the same inputs (bench.py Epoch, bench_configs.py), so the
sizes, workspaces, counters and tile lists the benchmarks time are the ones tested here.

  C2  100 coin instances x 100 SignatureShares + 100 G2 combines
  C3  1000 ciphertexts x 1000 DecryptionShares + 1000 G1 combines (uniform 1 % and the
      sender-concentrated 33 % pattern), plus a per-share-mode slice of 40 ciphertexts
  C4  64 coin instances x 10^4 SignatureShares + 64 combines of t = 3334 (property: statuses
      from the construction, combine == master_sk * H), on one context and on a two-slot node
  C5  one node's SyncKeyGen era at N = 1000: 1000 Parts (56 280-point commitments) and 10^6 Acks
"""
import numpy as np
import pytest

import bench
import bench_configs
from hbbft_amd import _native as N

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    c = N.Context(0)
    c.set_verify_mode(N.MODE_RLC)
    c.set_exact_below(0)
    yield c
    c.close()


@pytest.mark.timeout(300)
def test_c3_full_epoch_against_construction(ctx):
    ep = bench.Epoch(ctx, 1000, 1000, bench.SEED, 0.01)
    ep.step(ctx)
    mism, comb_ok, n_acc = ep.check(ctx)
    assert mism == 0 and comb_ok
    assert n_acc == int((ep.expected == N.ACCEPT).sum()) >= 1000 * 1000 - 10 * 1000 - 8
    # the group sums themselves are right (curve.h xadic_mul_sac8 in k_rlc_items): only the
    # tiles holding wrong shares fall back, about 2.3 k exact checks, not every share
    assert ctx.rlc_last_leaves() < 10000, ctx.rlc_last_leaves()
    # a second epoch through the same buffers (pipelined: combine k overlaps verification k+1)
    ep.step(ctx)
    mism, comb_ok, _ = ep.check(ctx)
    assert mism == 0 and comb_ok
    # per-share mode on a 40-ciphertext slice of the same shares equals the RLC decisions
    st_rlc, _, _ = ep.results(ctx)
    k = 40
    sh = ep.host_shares[:k * ep.n].reshape(-1)
    ctx.set_verify_mode(N.MODE_PER_SHARE)
    try:
        st_ps = ctx.verify_dec_shares(ep.keyset, ep.H[:96 * k], ep.w[:96 * k], [ep.n] * k,
                                      ep.idx[:k * ep.n], sh)
    finally:
        ctx.set_verify_mode(N.MODE_RLC)
    assert (st_ps == st_rlc[:k * ep.n]).all()
    ep.free(ctx)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("cts", [125, 250])
def test_c3_rank_slice_every_check_schedule(ctx, cts):
    """One rank's slice of a C3 epoch under strong scaling (1000 / 8 and 1000 / 4 ciphertexts
    of 1000 shares, 1 % wrong): the auto schedule (paired levels at this size), plain-first and
    both paired schedules all match the construction."""
    ep = bench.Epoch(ctx, 1000, cts, bench.SEED + cts, 0.01)
    try:
        for sched in (N.CHECK_AUTO, N.CHECK_PLAIN_FIRST, N.CHECK_PAIR_SUBS, N.CHECK_PAIR_LEAVES):
            ctx.set_check_schedule(sched)
            ep.step(ctx)
            mism, comb_ok, _ = ep.check(ctx)
            assert mism == 0 and comb_ok, sched
    finally:
        ctx.set_check_schedule(N.CHECK_AUTO)
    ep.free(ctx)


@pytest.mark.timeout(300)
def test_c3_sender_concentrated_33_percent(ctx):
    """f = 333 senders lie on every ciphertext: the first epoch finds them through failing
    groups, the second runs them as tracked senders; both match the construction."""
    ep = bench.Epoch(ctx, 1000, 1000, bench.SEED + 1, 0.0, "senders")
    for _ in range(2):
        ep.step(ctx)
        mism, comb_ok, n_acc = ep.check(ctx)
        assert mism == 0 and comb_ok
        assert n_acc == int((ep.expected == N.ACCEPT).sum()) >= 1000 * 1000 - 333 * 1000 - 8
    assert ctx.rlc_last_leaves() < 340 * 1000  # tracked: about the liars' shares only
    ep.free(ctx)


@pytest.mark.timeout(300)
def test_c2_full_against_construction(ctx):
    bench_configs.ctx_mode[0] = N.MODE_RLC
    out = bench_configs.bench_coins(ctx, "c2", 100, 100, 1, 0, 0.01)
    assert out["mismatches"] == 0 and out["combine_ok"]
    out = bench_configs.bench_coins(ctx, "c2", 100, 100, 1, 1, 0.0, "senders")
    assert out["mismatches"] == 0 and out["combine_ok"]


@pytest.mark.timeout(900)
def test_c4_full_64_instances_single_context_and_node(ctx):
    """BASELINE config 4 at full size (64 x 10^4 SignatureShares + 64 combines of t = 3334): on
    one context, and on a one-process node of two device slots (two contexts on this GPU:
    hbtc_node_*_dev with whole instances per slot, the path `bench_configs.py c4 --gpus N`
    runs on N GPUs).  Both equal the construction, and each other bit for bit (statuses,
    combined signatures, parities, combine statuses)."""
    bench_configs.ctx_mode[0] = N.MODE_RLC
    a = bench_configs.bench_coins(ctx, "c4", 10000, 64, 1, 0, 0.01, keep_arrays=True)
    assert a["mismatches"] == 0 and a["combine_ok"]
    # 10^4 tiles: the throughput form of k_sig_items (the two-addition x-adic loop, its table in
    # LDS); its group sums are right, so only tiles holding wrong shares reach exact checks
    assert ctx.rlc_last_leaves() < 64000, ctx.rlc_last_leaves()
    assert a["config"]["instances"] == 64 and a["config"]["t"] == 3334
    node = N.Node([0, 0])
    try:
        node.set_verify_mode(N.MODE_RLC)
        b = bench_configs.bench_coins(ctx, "c4", 10000, 64, 2, 1, 0.01, node=node, keep_arrays=True)
    finally:
        node.close()
    assert b["mismatches"] == 0 and b["combine_ok"]
    assert b["config"]["parallelism"].startswith("node: one process, 2 device slot(s) on 1 GPU(s)")
    for x, y in zip(a["_arrays"], b["_arrays"]):
        assert x.shape == y.shape and (x == y).all()


@pytest.mark.timeout(300)
@pytest.mark.parametrize("slots", [[0, 0, 0], [0, 0, 0, 0, 0, 0, 0, 0]])
def test_c2_node_slots_equal_single_context(ctx, slots):
    """C2 (100 x 100 SignatureShares, 33 % sender-concentrated) on a node of 3 and 8 slots (100
    instances cut unevenly by share count): equal to the single context bit for bit."""
    bench_configs.ctx_mode[0] = N.MODE_RLC
    a = bench_configs.bench_coins(ctx, "c2", 100, 100, 1, 0, 0.0, "senders", keep_arrays=True)
    node = N.Node(slots)
    try:
        node.set_verify_mode(N.MODE_RLC)
        b = bench_configs.bench_coins(ctx, "c2", 100, 100, 3, 1, 0.0, "senders", node=node,
                                      keep_arrays=True)
    finally:
        node.close()
    assert a["mismatches"] == 0 and b["mismatches"] == 0 and a["combine_ok"] and b["combine_ok"]
    for x, y in zip(a["_arrays"], b["_arrays"]):
        assert (x == y).all()


@pytest.mark.timeout(600)
def test_c5_full_era_against_construction(ctx):
    out = bench_configs.bench_skg(ctx, 1000, 1000, 4, 1, 0)
    assert out["mismatches"] == 0
    assert out["config"]["acks"] == 10 ** 6
