"""Sharding one epoch over ranks (hbbft_amd/shard.py, the plans of hbbft_amd/csrc/hbtc_node.cpp):
plan properties on ragged batches, then a world_size-2 gloo job that verifies and combines its
shard and merges with the same all-gather bench.py runs over RCCL.  The per-rank verification
and combines here are the C oracle (checker only), so the test covers the plan + merge logic
without a GPU; tests/test_gpu_parity.py runs the same plans through the HIP path."""
import os
import random
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from hbbft_amd import shard

R = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001


def _offsets(counts):
    off = np.zeros(len(counts) + 1, np.uint32)
    off[1:] = np.cumsum(counts)
    return off


CASES = [[7, 0, 13, 3, 9], [1000] * 10, [0, 0, 0], [5], [1, 2, 3, 4, 5, 6, 7, 8, 9], [10000], [],
         [0, 64, 0, 1, 0]]


@pytest.mark.parametrize("counts", CASES)
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_item_plan_partitions_every_item_once(counts, world):
    off = _offsets(counts)
    total = int(off[-1])
    covered = []
    prev_hi = 0
    for r in range(world):
        lo, hi, parent, sub = shard.item_plan(world, r, off)
        assert lo == prev_hi and lo <= hi
        prev_hi = hi
        assert sub[0] == 0 and sub[-1] == hi - lo and len(sub) == len(parent) + 1
        assert (np.diff(parent.astype(np.int64)) > 0).all()  # increasing, no empty sub-instance
        for s, k in enumerate(parent):
            a, b = lo + int(sub[s]), lo + int(sub[s + 1])
            assert b > a
            assert off[k] <= a and b <= off[k + 1]  # inside its parent instance
            covered.extend(range(a, b))
        assert hi - lo in (total // world, -(-total // world))  # equal slices
    assert prev_hi == total and covered == list(range(total))


@pytest.mark.parametrize("counts", CASES)
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_instance_plan_is_contiguous_and_balanced(counts, world):
    off = _offsets(counts)
    sl = shard.instance_slices(world, off)
    assert sl[0][0][0] == 0 and sl[-1][0][1] == len(counts)
    for r in range(world - 1):
        assert sl[r][0][1] == sl[r + 1][0][0]
    total = int(off[-1])
    biggest = max(counts) if counts else 0
    for (a, b), (lo, hi) in sl:
        assert (lo, hi) == (int(off[a]), int(off[b]))
        if total:  # no rank exceeds its fair share by more than one instance
            assert hi - lo <= -(-total // world) + biggest


def test_plan_rejects_bad_arguments():
    with pytest.raises(Exception):
        shard.item_plan(2, 2, _offsets([3]))
    with pytest.raises(Exception):
        shard.instance_plan(0, _offsets([3]))
    with pytest.raises(Exception):
        shard.item_plan(2, 0, np.array([1, 2], np.uint32))  # offsets[0] != 0


def _batch(seed):
    """A ragged 5-instance DecryptionShare batch with wrong shares and a bad encoding."""
    from oracle import cbaseline as C
    from oracle import bls12_381 as B
    rng = random.Random(seed)
    n, t = 7, 3
    coeffs = [rng.randrange(1, R) for _ in range(t)]
    sks = [sum(c * pow(i + 1, j, R) for j, c in enumerate(coeffs)) % R for i in range(n)]
    g1, g2 = B.g1_compress(B.G1_GEN), B.g2_compress(B.G2_GEN)
    pks = [C.g1_mul(g1, s) for s in sks]
    counts = [6, 0, 7, 3, 5]
    H, w, idx, shares, want = [], [], [], [], []
    for k, c in enumerate(counts):
        r, h = rng.randrange(1, R), rng.randrange(1, R)
        H.append(C.g2_mul(g2, h))
        w.append(C.g2_mul(g2, r * h % R))
        want.append(C.g1_mul(g1, coeffs[0] * r % R))
        senders = rng.sample(range(n), c)
        for j, i in enumerate(senders):
            sc = sks[i] * r % R
            if j == 1:
                sc = (sc + 1) % R  # wrong share
            sh = C.g1_mul(g1, sc)
            if k == 3 and j == 0:
                sh = bytes([sh[0] & 0x7F]) + sh[1:]  # invalid encoding
            idx.append(i)
            shares.append(sh)
    return dict(n=n, t=t, pks=pks, counts=counts, H=H, w=w, idx=idx, shares=shares, want=want)


def _verify(b, item, inst):
    """Checker: e(share, H) == e(pk_i, w) (threshold_decryption.rs:159) via the C oracle."""
    from oracle import cbaseline as C
    ok = C.pairing_eq(b["shares"][item], b["H"][inst], b["pks"][b["idx"][item]], b["w"][inst])
    return 2 if ok is None else (0 if ok else 1)


def _combine(b, st, off, k):
    from oracle import cbaseline as C
    acc = [j for j in range(int(off[k]), int(off[k + 1])) if st[j] == 0][:b["t"]]
    code, pt = C.combine(1, [b["idx"][j] for j in acc], [b["shares"][j] for j in acc], b["t"])
    return code, pt or bytes(48)


def _rank_main(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b = _batch(5)
    off = _offsets(b["counts"])
    # item plan: this rank's sub-instances, merged statuses
    lo, hi, parent, sub = shard.item_plan(world, rank, off)
    st_loc = np.zeros(hi - lo, np.int32)
    for s, k in enumerate(parent):
        for j in range(lo + int(sub[s]), lo + int(sub[s + 1])):
            st_loc[j - lo] = _verify(b, j, int(k))
    lens = [shard.item_plan(world, r, off)[1] - shard.item_plan(world, r, off)[0] for r in range(world)]
    st_all = shard.gather_slices(dist, torch.from_numpy(st_loc), lens).numpy()
    # instance plan: this rank's combines over the merged statuses, merged points
    sl = shard.instance_slices(world, off)
    a, bb = sl[rank][0]
    pts = np.zeros((bb - a, 48), np.uint8)
    codes = np.zeros(bb - a, np.int32)
    for k in range(a, bb):
        codes[k - a], p = _combine(b, st_all, off, k)
        pts[k - a] = np.frombuffer(p, np.uint8)
    lc = [y - x for (x, y), _ in sl]
    pts_all = shard.gather_slices(dist, torch.from_numpy(pts), lc).numpy()
    codes_all = shard.gather_slices(dist, torch.from_numpy(codes), lc).numpy()
    np.savez(os.path.join(out_dir, "r%d.npz" % rank), st=st_all, pts=pts_all, codes=codes_all)
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.timeout(300)
def test_two_rank_gloo_shard_and_merge_equals_whole_batch(tmp_path):
    pytest.importorskip("oracle.cbaseline")
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    b = _batch(5)
    off = _offsets(b["counts"])
    st = np.array([_verify(b, j, k) for k in range(len(b["counts"]))
                   for j in range(int(off[k]), int(off[k + 1]))], np.int32)
    assert sorted(set(st.tolist())) == [0, 1, 2]
    whole = [_combine(b, st, off, k) for k in range(len(b["counts"]))]
    for r in range(world):
        got = np.load(tmp_path / ("r%d.npz" % r))
        assert (got["st"] == st).all()
        assert got["codes"].tolist() == [c for c, _ in whole]
        assert [bytes(p) for p in got["pts"]] == [p for _, p in whole]
    # the combines that succeed reproduce the master key's decryption share
    for k, (code, p) in enumerate(whole):
        if code == 0:
            assert p == b["want"][k]
