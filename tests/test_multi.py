"""Multi-process (world size 2, gloo on CPU) checks of the sharded path: the
shard boundaries partition the batch, per-rank results concatenate to the
single-process results, and the counter all-reduce equals the whole-batch
counters. The per-rank compute here is the CPU oracle (no GPU on this host);
the GPU box runs the same sharding with the HIP kernel (tests/test_gpu_multi.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import libpnet_amd as lp
from libpnet_amd import shard
from oracle import coracle

WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def counters_of(rec, lens):
    st = rec["status"].astype(np.int64)
    return np.array([len(st), int(lens.astype(np.int64).sum()), int(((st & 3) == 1).sum()),
                     int(((st & 3) == 2).sum()),
                     int((((st & 3) == 1) & ((st & 0x40) == 0) & ((st & 0x100) == 0)).sum()),
                     int((((st & 0x200) != 0) & ((st & 0x400) == 0)).sum()),
                     int(((st & (0x20 | 0x40 | 0x80 | 0x8000)) != 0).sum()),
                     int(((st & (0x800 | 0x1000)) != 0).sum())], dtype=np.int64)


def _worker(rank, port, n, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    w = lp.synth.make("imix", n, seed=77)
    lo, hi = shard.shard_by_bytes(w.lengths, WORLD, rank)
    rec = coracle.rx_batch(w.buf, hi - lo, offsets=w.offsets[lo:hi], lengths=w.lengths[lo:hi])
    ctr = torch.from_numpy(counters_of(rec, w.lengths[lo:hi]))
    shard.all_reduce_counters(ctr)
    tmax = shard.all_reduce_max(float(rank + 1), "cpu")
    gathered = [None] * WORLD
    dist.all_gather_object(gathered, (lo, hi, rec.tobytes()))
    if rank == 0:
        out.put((ctr.numpy().tolist(), tmax, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_shards_match_single_process():
    n = 20000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, n, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    ctr, tmax, gathered = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = lp.synth.make("imix", n, seed=77)
    full = coracle.rx_batch(w.buf, n, offsets=w.offsets, lengths=w.lengths)
    assert ctr == counters_of(full, w.lengths).tolist()
    assert tmax == float(WORLD)
    spans = sorted((lo, hi) for lo, hi, _ in gathered)
    assert spans[0][0] == 0 and spans[-1][1] == n and spans[0][1] == spans[1][0]
    cat = np.concatenate([np.frombuffer(b, dtype=coracle.REC_DTYPE) for _, _, b in sorted(gathered)])
    assert (cat == full).all()


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_shard_partitions(world):
    rng = np.random.default_rng(world)
    lengths = rng.choice([64, 576, 1500], size=10007, p=[7 / 12, 4 / 12, 1 / 12]).astype(np.uint32)
    for fn in (lambda r: shard.shard_by_index(len(lengths), world, r),
               lambda r: shard.shard_by_bytes(lengths, world, r)):
        spans = [fn(r) for r in range(world)]
        assert spans[0][0] == 0 and spans[-1][1] == len(lengths)
        assert all(spans[i][1] == spans[i + 1][0] for i in range(world - 1))
    tot = int(lengths.sum())
    for r in range(world):
        lo, hi = shard.shard_by_bytes(lengths, world, r)
        assert abs(int(lengths[lo:hi].sum()) - tot / world) <= 1500
