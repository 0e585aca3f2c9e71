"""Multi-process sharding with the HIP kernel (SURVEY.md §4 implication 4, §8(e)):
two ranks, one process each, on this box's GPU (a 1-GPU box stands in for two
devices; the bench's N-GPU runs use RCCL). Each rank uploads and processes its
byte-balanced slice of an IMIX batch through the C-ABI, the counter vectors are
all-reduced, and the concatenated per-rank records equal the oracle's over the
whole batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
WORLD = 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, n, q):
    import libpnet_amd as lp
    from libpnet_amd import shard
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=WORLD)
    try:
        torch.cuda.set_device(0)
        w = lp.synth.make("imix", n, seed=91, corrupt_ppm=20000)
        lo, hi = shard.shard_by_bytes(w.lengths, WORLD, rank)
        b0 = int(w.offsets[lo])
        b1 = int(w.offsets[hi - 1]) + int(w.lengths[hi - 1])
        data = torch.from_numpy(np.concatenate([w.buf[b0:b1], np.zeros(32, np.uint8)])).to("cuda:0")
        offs = torch.from_numpy((w.offsets[lo:hi] - b0).view(np.int64)).to("cuda:0")
        lens = torch.from_numpy(w.lengths[lo:hi].view(np.int32)).to("cuda:0")
        res = lp.rx_process(data, offsets=offs, lengths=lens, columns=lp.ALL_COLUMNS)
        torch.cuda.synchronize()
        ctr = res.counters.cpu()
        shard.all_reduce_counters(ctr)
        recs = {c: v for c, v in res.numpy().items()}
        gathered = [None] * WORLD
        dist.all_gather_object(gathered, (lo, hi, recs))
        if rank == 0:
            q.put((ctr.numpy().view(np.uint64).tolist(), gathered))
        dist.barrier()
    finally:
        dist.destroy_process_group()


def test_two_ranks_gpu_shards_match_whole_batch_oracle():
    import libpnet_amd as lp
    from oracle import coracle
    n = 60000
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, port, n, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    ctr, gathered = q.get(timeout=100)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    w = lp.synth.make("imix", n, seed=91, corrupt_ppm=20000)
    full = coracle.rx_batch(w.buf, n, offsets=w.offsets, lengths=w.lengths)
    spans = sorted((lo, hi) for lo, hi, _ in gathered)
    assert spans[0][0] == 0 and spans[-1][1] == n and spans[0][1] == spans[1][0]
    for lo, hi, recs in gathered:
        for c, v in recs.items():
            assert np.array_equal(v, full[c][lo:hi]), (lo, c)
    assert ctr[0] == n and ctr[1] == int(w.lengths.astype(np.int64).sum())
    assert ctr[4] == w.expect["ip_bad"] and ctr[5] == w.expect["l4_bad"]


def test_bench_two_ranks_one_gpu():
    """The driver's `python bench.py --gpus 2` end to end with the HIP kernel:
    the parent starts two ranks (torchrun child), both run on this box's one GPU
    (gloo stands in for RCCL: two ranks cannot share one device under RCCL), and
    rank 0's single line reports n_gpus 2 with every planted corruption counted."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PNETGPU_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3",
                        "--warmup", "1", "--frames-scale", "0.01", "--workloads", "udp64,imix", "--no-cpu",
                        "--no-e2e", "--no-extra"], cwd=root, env=env, capture_output=True, text=True, timeout=100)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 2 and line["counters_ok"] is True
    assert line["collective"] == {"backend": "gloo", "world_size": 2, "library": "gloo"}
    assert line["workloads"]["imix"]["counters_ok"] is True
    assert line["config"]["frames_scale"] == 0.01
    # one global batch, sharded: the two ranks' frames add up to it
    assert line["config"]["global_batch_frames"] == 2 * int((1 << 24) * 0.01)
    assert line["config"]["parallelism"] == "shard_by_index x2"
    assert line["workloads"]["imix"]["counters_ok"] is True


def test_bench_four_ranks_one_gpu():
    """A rehearsal of the driver's scaling run on the 1-GPU box: `bench.py --gpus 4`
    (gloo standing in for RCCL) over udp64 and IMIX at a small frame scale. The
    IMIX cuts come from rank 0's prefix sum (broadcast), the four shards add up
    to the global batch, every planted corruption is counted, and the line
    carries each workload's per-rank kernel-time spread."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PNETGPU_BENCH_BACKEND"] = "gloo"
    p = subprocess.run([sys.executable, "-u", os.path.join(root, "bench.py"), "--gpus", "4", "--steps", "3",
                        "--warmup", "1", "--frames-scale", "0.002", "--workloads", "udp64,imix", "--no-cpu",
                        "--no-e2e", "--no-extra"], cwd=root, env=env, capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [json.loads(ln) for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout
    line = lines[0]
    assert line["n_gpus"] == 4 and line["counters_ok"] is True
    assert line["collective"] == {"backend": "gloo", "world_size": 4, "library": "gloo"}
    assert line["config"]["global_batch_frames"] == 4 * int((1 << 24) * 0.002)
    im = line["workloads"]["imix"]
    assert im["counters_ok"] is True
    assert im["frames_per_step"] == 4 * int((1 << 22) * 0.002)
    for w in ("udp64", "imix"):
        r = line["workloads"][w]
        assert 0 < r["kernel_ms_min"] <= r["kernel_avg_ms"] <= r["kernel_ms_max"]


def _rccl_worker(port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("nccl", rank=0, world_size=1)   # nccl = RCCL on ROCm
    try:
        import libpnet_amd as lp
        from libpnet_amd import shard
        lengths = lp.synth.lengths("imix", 100003, 7)
        cuts = shard.broadcast_byte_cuts(lambda: lengths, 1, 0, device=dev)
        ctr = torch.arange(8, dtype=torch.int64, device=dev)
        shard.all_reduce_counters(ctr)
        mx = shard.all_reduce_max(2.5, dev)
        mn_mx = shard.all_reduce_min_max(1.25, dev)
        q.put((cuts, ctr.cpu().tolist(), mx, mn_mx, dist.get_backend()))
    finally:
        dist.destroy_process_group()


def test_rccl_collectives_one_rank():
    """The RCCL (`nccl` backend) code path of the multi-GPU bench on this box's
    one GPU: the byte-cut broadcast, the counter all-reduce and the MIN/MAX
    time reductions run through RCCL on device tensors (the 8-GPU run uses the
    same calls with 8 ranks; two ranks cannot share one device under RCCL)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_worker, args=(_free_port(), q))
    p.start()
    cuts, ctr, mx, mn_mx, backend = q.get(timeout=100)
    p.join(timeout=60)
    assert p.exitcode == 0
    assert backend == "nccl"
    assert cuts == (0, 100003)
    assert ctr == list(range(8)) and mx == 2.5 and mn_mx == (1.25, 1.25)
