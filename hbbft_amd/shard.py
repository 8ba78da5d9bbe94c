"""Sharding one node's epoch over several GPUs, one process per GPU (strong scaling).

hbbft runs one process per node (/root/reference/src/messaging.rs:188) with at most
max_future_epochs = 3 epochs in flight (src/honey_badger/builder.rs:37), so the GPUs of a node
split ONE epoch's share batch rather than running separate epochs.  The plans are the native
node's (hbtc_shard_items / hbtc_shard_instances in hbbft_amd/csrc/hbtc_node.cpp, so a
multi-process job and the single-process hbtc_node_* calls cut a batch identically):

  instance plan  rank r takes whole instances [first[r], first[r+1]), balanced by share count;
                 its verification AND its combines stay on its GPU (the combine reads the
                 verdicts of the same instances), so the data path has no exchange.
  item plan      equal contiguous item slices; an instance crossing a cut is verified as one
                 sub-instance per side (the RLC groups are tiles inside an instance).  Used when
                 there are fewer instances than ranks (one N = 10^4 coin over 8 GPUs).

The merge is the one collective of the north star: an all-gather of every rank's verdicts
(int32 statuses) and combined points, padded to the longest rank's slice
(`gather_slices`).  It works on any torch.distributed backend: RCCL (`nccl`) over xGMI on the
GPU box with device tensors, gloo with host tensors in the CPU tests.
"""
import ctypes

import numpy as np

from . import _native as N


def instance_plan(world, offsets):
    """first[r] .. first[r+1]: rank r's instances (hbtc_shard_instances)."""
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    first = np.zeros(world + 1, np.uint32)
    rc = N.load().hbtc_shard_instances(world, off.size - 1, N._ptr(off), N._ptr(first))
    if rc != 0:
        raise N.HbtcError("hbtc_shard_instances: bad arguments (%d)" % rc)
    return first


def item_plan(world, rank, offsets):
    """Rank `rank`'s verification slice: (lo, hi, parent, sub_offsets) (hbtc_shard_items)."""
    off = np.ascontiguousarray(offsets, dtype=np.uint32)
    n_inst = off.size - 1
    lo, hi, n_sub = N._U32(), N._U32(), N._U32()
    parent = np.zeros(max(n_inst, 1), np.uint32)
    sub = np.zeros(n_inst + 1, np.uint32)
    rc = N.load().hbtc_shard_items(world, rank, n_inst, N._ptr(off), ctypes.byref(lo), ctypes.byref(hi),
                                   ctypes.byref(n_sub), N._ptr(parent), N._ptr(sub))
    if rc != 0:
        raise N.HbtcError("hbtc_shard_items: bad arguments (%d)" % rc)
    return lo.value, hi.value, parent[:n_sub.value].copy(), sub[:n_sub.value + 1].copy()


def instance_slices(world, offsets):
    """Per rank: (instance range, item range) of the instance plan."""
    first = instance_plan(world, offsets)
    off = np.asarray(offsets, dtype=np.int64)
    return [((int(first[r]), int(first[r + 1])), (int(off[first[r]]), int(off[first[r + 1]])))
            for r in range(world)]


def gather_slices(dist, local, lengths, out=None):
    """All-gather rank slices of different lengths into one array in rank order.

    `local` is this rank's slice (a torch tensor, first dim = its length), `lengths[r]` every
    rank's length.  Each rank sends its slice padded to max(lengths) (one all_gather_into_tensor
    over the backend's stream: RCCL over xGMI for device tensors); the result is the
    concatenation of the unpadded slices, i.e. the whole batch's array."""
    import torch
    if local.is_cuda and dist.get_backend() == "gloo":  # gloo gathers host tensors
        merged = gather_slices(dist, local.cpu(), lengths).to(local.device)
        if out is not None:
            out.copy_(merged)
            return out
        return merged
    world = len(lengths)
    m = max(lengths) if lengths else 0
    rest = tuple(local.shape[1:])
    if local.shape[0] != m:
        pad = torch.zeros((m,) + rest, dtype=local.dtype, device=local.device)
        pad[:local.shape[0]] = local
        local = pad
    buf = torch.empty((world * m,) + rest, dtype=local.dtype, device=local.device)
    dist.all_gather_into_tensor(buf, local)
    parts = [buf[r * m:r * m + lengths[r]] for r in range(world)]
    merged = torch.cat(parts) if parts else buf[:0]
    if out is not None:
        out.copy_(merged)
        return out
    return merged
