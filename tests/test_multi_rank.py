"""The N>1 bench path on CPU: world_size-2 gloo (the driver runs bench.py under
torch.distributed.run, one rank per GPU).  Checks the weak-scaling contract: every rank gets its
own epoch shard (distinct seeds, no data-path collective) and the job time is the barrier-
bracketed MAX over ranks, on every rank."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, out_dir):
    import torch.distributed as dist

    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    elapsed = bench.max_over_ranks(1.5 + rank, dist)
    with open(os.path.join(out_dir, "r%d" % rank), "w") as fh:
        fh.write("%r %d" % (elapsed, bench.rank_seed(rank)))
    dist.destroy_process_group()


@pytest.mark.timeout(120)
def test_two_rank_gloo_max_time_and_disjoint_shards(tmp_path):
    world = 2
    mp.spawn(_rank_main, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    res = [open(tmp_path / ("r%d" % r)).read().split() for r in range(world)]
    assert [float(e) for e, _ in res] == [1.5 + world - 1] * world
    seeds = [int(s) for _, s in res]
    assert len(set(seeds)) == world


def test_single_rank_time_is_local():
    import bench
    assert bench.max_over_ranks(0.25, None) == 0.25
