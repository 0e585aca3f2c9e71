"""Multi-GPU sharding of frame batches.

Frames are independent, so a batch shards by frame index with no data-path
exchange: each rank (one process per GPU) processes its contiguous slice and
writes its own result slice. The only collective is one all-reduce of the
uint64 counter vector at the end (RCCL over xGMI on GPUs, gloo on CPU), the
"final throughput reduction". This mirrors the reference's only multi-worker
mechanism, PACKET_FANOUT socket sharding (pnet_datalink/src/linux.rs:156-200),
but partitions a resident batch instead of a socket's arrival stream.
"""
import numpy as np
import torch


def shard_by_index(n, world, rank):
    """[lo, hi) frame range of `rank` when n frames are split evenly by count."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    return n * rank // world, n * (rank + 1) // world


def byte_cuts(lengths, world):
    """The world + 1 frame-index cut points of a byte-balanced split (rank k owns
    [cuts[k], cuts[k + 1])): cut k is the first frame index whose byte prefix
    reaches k/world of the total, so every rank streams about the same number of
    bytes. One prefix sum for all ranks."""
    lengths = np.asarray(lengths, dtype=np.uint64)
    n = lengths.size
    if n == 0:
        return [0] * (world + 1)
    prefix = np.cumsum(lengths, dtype=np.uint64)
    total = int(prefix[-1])
    cuts = [0]
    for k in range(1, world):
        cuts.append(min(int(np.searchsorted(prefix, (total * k + world - 1) // world, side="left")) + 1, n))
    cuts.append(n)
    return cuts


def shard_by_bytes(lengths, world, rank):
    """[lo, hi) frame range of `rank` with the frame BYTES split evenly (IMIX)."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    cuts = byte_cuts(lengths, world)
    return cuts[rank], cuts[rank + 1]


def broadcast_byte_cuts(lengths_fn, world, rank, device=None, group=None):
    """[lo, hi) of `rank` under shard_by_bytes, with the global length vector
    built and prefix-summed on rank 0 ONLY (lengths_fn() is called there) and
    the world + 1 cut points broadcast: no other rank holds the global vector
    (2^25 entries for 8 ranks of the IMIX bench). Without an initialised
    process group this is shard_by_bytes on the local vector."""
    dist = torch.distributed.is_available() and torch.distributed.is_initialized()
    if not dist:
        return shard_by_bytes(lengths_fn(), world, rank)
    cuts = torch.zeros(world + 1, dtype=torch.int64, device=device)
    if rank == 0:
        cuts.copy_(torch.tensor(byte_cuts(lengths_fn(), world), dtype=torch.int64))
    torch.distributed.broadcast(cuts, src=0, group=group)
    return int(cuts[rank].item()), int(cuts[rank + 1].item())


def all_reduce_min_max(value, device, group=None):
    """(min, max) of a float over all ranks (per-rank kernel times: shard imbalance)."""
    t = torch.tensor([float(value), -float(value)], dtype=torch.float64, device=device)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
    return -float(t[1].item()), float(t[0].item())


def all_reduce_counters(counters, group=None):
    """Sum an int64 counter tensor over all ranks (in place) and return it."""
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.all_reduce(counters, op=torch.distributed.ReduceOp.SUM, group=group)
    return counters


def all_reduce_max(value, device, group=None):
    """Max of a float over all ranks (the wall time of a weak-scaling step)."""
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    if torch.distributed.is_available() and torch.distributed.is_initialized():
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX, group=group)
    return float(t.item())
