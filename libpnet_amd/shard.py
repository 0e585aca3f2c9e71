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


def shard_by_bytes(lengths, world, rank):
    """[lo, hi) frame range of `rank` with the frame BYTES split evenly (IMIX).

    Boundaries are the first frame index whose byte prefix reaches k/world of
    the total, so every rank streams about the same number of bytes."""
    if not (0 <= rank < world):
        raise ValueError("rank out of range")
    lengths = np.asarray(lengths, dtype=np.uint64)
    n = lengths.size
    if n == 0:
        return 0, 0
    prefix = np.cumsum(lengths, dtype=np.uint64)
    total = int(prefix[-1])

    def cut(k):
        if k == 0:
            return 0
        if k == world:
            return n
        return int(np.searchsorted(prefix, (total * k + world - 1) // world, side="left")) + 1

    return min(cut(rank), n), min(cut(rank + 1), n)


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
