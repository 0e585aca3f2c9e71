#!/usr/bin/env python3
"""Benchmark: device-resident receive-path throughput (parse + verify) on MI355X.

BASELINE.json metric: "device-resident Mpkts/s & GB/s, checksum+parse, 64B & 1500B,
1/2/4/8 GPU". One step = one pnetgpu_rx_process launch over a resident batch:
  primary   configs[1]  64-B Eth/IPv4/UDP, 2^24 frames (1 GiB) per GPU  -> `value`
  secondary configs[2]  1500-B Eth/IPv4/TCP, 2^20 frames (1.5 GiB) per GPU
Both write the full IPv4 record (status, both checksums, ethertype, proto, ttl,
L4 offset/length, ports, addresses) plus counters. Multi-GPU: one process per
GPU (torchrun), each with its own shard (weak scaling, no data-path collective);
RCCL only all-reduces the counters once at the end and takes the max time.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--no-cpu] [--no-e2e] [--no-extra]
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

# libpnet_amd (the HIP library) is imported by main() only after the launcher
# decision: a `--gpus N` parent that starts the ranks never loads it
lp = shard = None

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (/opt/skills/guides/MI355X_MICROARCH.md:36)
METRIC = "device-resident Mpkts/s & GB/s, checksum+parse, 64B & 1500B, 1/2/4/8 GPU"
WORKLOADS = {
    "udp64": {"n": 1 << 24, "desc": "configs[1]: 64B UDP/IPv4/Ethernet, checksum verify + header extract, "
                                    "device-resident batch"},
    "tcp1500": {"n": 1 << 20, "desc": "configs[2]: 1500B TCP/IPv4/Ethernet, full-MTU ones-complement sum over "
                                      "pseudo-header+payload"},
    # north_star states its >=70 % target on "64 B and 1500 B UDP/IPv4" at 1 GPU:
    # the rs_sender.rs:54-72 frame at full MTU (udp.rs:34-56 over 1466 B)
    "udp1500": {"n": 1 << 20, "desc": "north_star: 1500B UDP/IPv4/Ethernet (1458 data bytes), checksum verify + "
                                      "header extract, device-resident batch"},
    # BASELINE's 8-GPU configs, per-GPU shard sizes (weak scaling); secondary lines
    "imix": {"n": 1 << 22,
             "desc": "configs[3]: IMIX 64/576/1500B 7:4:1 Eth/IPv4/{UDP,TCP,ICMP}, descriptor mode, per-GPU shard"},
    "udp6_jumbo": {"n": 1 << 17,
                   "desc": "configs[4]: 9000B IPv6/UDP jumbo frames, IPv6 pseudo-header checksum, per-GPU shard"},
    # configs[1]'s frames with the verify-only record (status + both computed
    # checksums, R = 6 B/frame; SURVEY.md §8(d) priced the target with R = 8):
    # the same kernel, a consumer that reads no extracted fields
    "imix_verify": {"n": 1 << 22, "synth": "imix", "columns": ("status", "ip_csum", "l4_csum"),
                    "desc": "configs[3] frames, checksum verify only (status + ip_csum + l4_csum columns)"},
    "udp64_verify": {"n": 1 << 24, "synth": "udp64", "columns": ("status", "ip_csum", "l4_csum"),
                     "desc": "configs[1] frames, checksum verify only (status + ip_csum + l4_csum columns)"},
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Shard:
    """One workload resident on this rank's GPU, with its result buffers."""

    def __init__(self, name, n, seed, device, first=0):
        self.name, self.n, self.first = name, n, first
        cfg = WORKLOADS.get(name, {})
        columns = cfg.get("columns", lp.IPV4_COLUMNS)
        # frames [first, first + n) of the global batch `seed` defines
        w = lp.synth.make(cfg.get("synth", name), n, seed=seed, corrupt_ppm=10000, first=first)
        self.w = w
        self.data = torch.from_numpy(w.buf).to(device)
        self.offsets = self.lengths = None
        self.flags = 0
        self.desc_bytes = 0
        if not w.stride:
            # compact descriptors (u32 offset + u16 length, PNETGPU_DESC_COMPACT) when
            # they can describe the batch, else u64 + u32
            if w.buf.size <= 0xFFFFFFFF and int(w.lengths.max()) <= 0xFFFF:
                self.offsets = torch.from_numpy(w.offsets.astype(np.uint32).view(np.int32)).to(device)
                self.lengths = torch.from_numpy(w.lengths.astype(np.uint16).view(np.int16)).to(device)
                self.flags, self.desc_bytes = lp.DESC_COMPACT, 6
            else:
                self.offsets = torch.from_numpy(w.offsets.view(np.int64)).to(device)
                self.lengths = torch.from_numpy(w.lengths.view(np.int32)).to(device)
                self.desc_bytes = 12
        self.res = lp.RxResult(n, device, columns, counters=True)
        self.frame_bytes = w.expect["bytes"]
        self.result_bytes = lp.column_bytes(columns)
        # algorithmic bytes per launch: frames read once + result columns written + descriptors
        self.alg_bytes = self.frame_bytes + n * (self.result_bytes + self.desc_bytes)

    def step(self, stream):
        if self.w.stride:
            lp.rx_process(self.data, stride=self.w.stride, frame_len=self.w.frame_len, n_frames=self.n,
                          out=self.res, stream=stream)
        else:
            lp.rx_process(self.data, offsets=self.offsets, lengths=self.lengths, out=self.res, stream=stream,
                          flags=self.flags)


def time_shard(sh, steps, warmup, stream, dist_on):
    """Wall time of exactly `steps` back-to-back launches, and the kernel's average
    launch duration from one HIP event pair on the launch stream around the same
    region (elapsed / steps: includes the few-us launch gaps, so it is an upper
    bound on the kernel time). Per-launch event pairs are not used: every timed
    event record adds ~6 us to the interval around the 64-B kernel (a 2.5 %
    inflation measured on MI355X, tools/launch_gap.py)."""
    for _ in range(warmup):
        sh.step(stream)
    stream.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    if dist_on:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    a.record(stream)
    for _ in range(steps):
        sh.step(stream)
    b.record(stream)
    stream.synchronize()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if dist_on:
        torch.distributed.barrier()
    return wall, a.elapsed_time(b) / steps


def check_counters(sh):
    """Size-independent property: every planted corruption found, nothing else."""
    sh.res.counters.zero_()
    sh.step(torch.cuda.current_stream())
    torch.cuda.synchronize()
    c = sh.res.counter_dict()
    ok = (c["frames"] == sh.n and c["bytes"] == sh.w.expect["bytes"] and c["ip_csum_bad"] == sh.w.expect["ip_bad"]
          and c["l4_csum_bad"] == sh.w.expect["l4_bad"] and c["malformed"] == 0 and c["unknown"] == 0)
    return ok, c


def host_cpu():
    """The host the CPU baseline ran on (record nproc and the model)."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for ln in f:
                if ln.startswith("model name"):
                    model = ln.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = None
    return {"cpu_model": model, "host_cpus": os.cpu_count(), "usable_cpus": usable}


def usable_cpus():
    try:
        return len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        return os.cpu_count() or 1


def cgroup_cpu_quota():
    """CPUs' worth of time the cgroup grants (cpu.max), None if unlimited/unknown."""
    try:
        with open("/sys/fs/cgroup/cpu.max") as fh:
            q, p = fh.read().split()[:2]
        return None if q == "max" else round(int(q) / int(p), 2)
    except (OSError, ValueError):
        return None


def _timed_reps(fn, target_s):
    """Rate of fn(reps): one warm-up pass (page faults, caches), one timed pass to
    size the sample, then one timed run of about target_s seconds."""
    fn(1)
    t = time.perf_counter()
    fn(1)
    t1 = max(time.perf_counter() - t, 1e-4)
    reps = max(1, min(1000, int(target_s / t1)))
    t = time.perf_counter()
    fn(reps)
    return reps, time.perf_counter() - t


def cpu_baseline(sh, target_s=3.0):
    """The oracle (scalar C restatement, 'port') timed on this host: all usable
    cores (`value`, persistent threads over static shards), 16 threads and one
    core, over a bounded sample of the same batch."""
    from oracle import coracle  # checker / baseline only
    w = sh.w
    n = min(sh.n, 1 << 22)
    out = np.zeros(n, dtype=coracle.REC_DTYPE)
    kw = dict(stride=w.stride, frame_len=w.frame_len) if w.stride else dict(offsets=w.offsets[:n],
                                                                              lengths=w.lengths[:n])
    per_frame_bytes = w.expect["bytes"] / sh.n
    quota = cgroup_cpu_quota()
    counts = [("all", usable_cpus())]
    if quota and int(quota) < usable_cpus():
        counts.append(("quota", max(1, int(quota))))     # the cgroup's share of the CPUs
    counts += [("16", 16), ("1", 1)]
    rates = {}
    for label, nthreads in counts:
        nn = n if nthreads > 1 else min(n, 1 << 18)
        kwn = kw if w.stride else dict(offsets=w.offsets[:nn], lengths=w.lengths[:nn])
        reps, el = _timed_reps(lambda r: coracle.rx_batch_reps(w.buf, nn, nthreads=nthreads, reps=r, out=out[:nn],
                                                               **kwn), target_s if label == "all" else target_s / 2)
        rates[label] = (nn * reps / el / 1e6, nthreads, reps, el, nn)
    # `value` = the best of the thread counts (every usable CPU by affinity, the
    # cgroup quota, 16, 1): with a CPU quota below the affinity mask, one thread
    # per affinity CPU oversubscribes the quota and runs slower than the quota's
    # worth of threads; every count's rate is kept beside it
    best = max(rates, key=lambda k: rates[k][0])
    mpps, nthreads, reps, el, nn = rates[best]
    return {"value": round(mpps, 2), "unit": "Mpkts/s", "cores": nthreads, "kind": "port",
            "value_all_usable_cpus": round(rates["all"][0], 2), "threads_all_usable_cpus": rates["all"][1],
            **({"value_quota_threads": round(rates["quota"][0], 2)} if "quota" in rates else {}),
            "value_16threads": round(rates["16"][0], 2), "value_1core": round(rates["1"][0], 2),
            **host_cpu(), "cgroup_cpu_quota": quota,
            "gbps": round(mpps * 1e6 * per_frame_bytes / 1e9, 2),
            "sample": f"first {nn} frames of the same {sh.name} batch x{reps} passes ({el:.1f} s wall, "
                      f"{nthreads} threads (best of {', '.join(str(c) for _, c in counts)}), persistent threads "
                      f"over static index shards; oracle/pnet_oracle.c scalar per-frame restatement writing its "
                      f"120-B record)"}


def config0_block(steps, warmup, device):
    """BASELINE configs[0] (benches/rs_sender.rs + rs_receiver.rs, CPU plumbing):
    1M rs_sender frames built + checksummed on the CPU (the oracle's restatement
    of build_udp4_packet, rs_sender.rs:25-72) on one core and on every usable
    core; their receive + verify on the CPU over an in-memory ring (the
    dummy.rs:133-153 receiver hands each frame over without a copy); and the GPU
    legs over the same 1M frames, device-resident: tx_fill_checksums on frames
    whose checksum fields are zero, then rx_process. The loopback AF_PACKET
    send/receive needs CAP_NET_RAW, which the GPU box does not grant."""
    from oracle import coracle  # CPU legs only
    n = 1 << 20
    buf = np.zeros(64 * n + 32, dtype=np.uint8)
    out = {"frames": n, "frame_bytes": 64}
    for label, nthreads in (("1core", 1), ("all", usable_cpus())):
        reps, el = _timed_reps(lambda r: coracle.rs_sender_build(n, nthreads=nthreads, reps=r, buf=buf), 2.0)
        out[f"cpu_build_checksum_{label}_mframes_s"] = round(n * reps / el / 1e6, 2)
    rec = np.zeros(n, dtype=coracle.REC_DTYPE)
    for label, nthreads in (("1core", 1), ("all", usable_cpus())):
        reps, el = _timed_reps(lambda r: coracle.rx_batch_reps(buf, n, stride=64, frame_len=64, nthreads=nthreads,
                                                               reps=r, out=rec), 2.0)
        out[f"cpu_receive_verify_{label}_mframes_s"] = round(n * reps / el / 1e6, 2)
    out["cpu_threads_all"] = usable_cpus()
    ok = (rec["status"] & 0x0500) == 0x0500
    out["cpu_frames_verified"] = int(ok.sum())
    # GPU legs: the same frames with both checksum fields cleared, filled on the GPU
    blank = buf.reshape(-1)[: 64 * n].reshape(n, 64).copy()
    blank[:, 24:26] = 0
    blank[:, 40:42] = 0
    d = torch.from_numpy(np.concatenate([blank.reshape(-1), np.zeros(32, np.uint8)])).to(device)
    dcopy = d.clone()
    st = lp.RxResult(n, device, ("status",), counters=False)
    stream = torch.cuda.Stream(device)
    ms_tx = time_launches(lambda s: lp.tx_fill_checksums(d, stride=64, frame_len=64, n_frames=n, out=st, stream=s),
                          steps, warmup, stream)
    res = lp.RxResult(n, device, lp.IPV4_COLUMNS, counters=True)
    ms_rx = time_launches(lambda s: lp.rx_process(d, stride=64, frame_len=64, n_frames=n, out=res, stream=s),
                          steps, warmup, stream)
    # the filled frames equal the CPU-built ones byte for byte (every checksum the sender computed)
    d.copy_(dcopy)
    torch.cuda.synchronize()          # the restore (current stream) before the fill (`stream`)
    lp.tx_fill_checksums(d, stride=64, frame_len=64, n_frames=n, out=st, stream=stream)
    stream.synchronize()
    out["gpu_tx_fill_identical_to_cpu_build"] = bool(np.array_equal(d[: 64 * n].cpu().numpy(), buf[: 64 * n]))
    out["gpu_tx_fill_mframes_s"] = round(n / (ms_tx * 1e-3) / 1e6, 1)
    out["gpu_tx_fill_kernel_ms"] = round(ms_tx, 4)
    out["gpu_rx_verify_mframes_s"] = round(n / (ms_rx * 1e-3) / 1e6, 1)
    out["gpu_rx_verify_kernel_ms"] = round(ms_rx, 4)
    out["note"] = ("CPU: oracle/pnet_oracle.c (rs_sender_build = rs_sender.rs:25-72 per frame; receive = the "
                   "packetdump.rs chain per frame, dummy-ring hand-over); GPU: kernel time over 2^20 resident "
                   "frames (a 64-MiB batch, L2/MALL-resident: not an HBM figure); the loopback AF_PACKET "
                   "send/receive needs CAP_NET_RAW, which the GPU box does not grant, and its user namespaces "
                   "are refused (unshare: ENOSPC); tests/test_netns_loopback.py runs that leg where allowed")
    return out


def _link(frames, el, up, down):
    """The PCIe link's share of an e2e line: bytes each frame moves up (frame +
    descriptors) and down (its record columns), and the link rate that implies,
    so lines with different records compare on the same link."""
    return {"link_bytes_per_frame": {"up": round(up, 2), "down": round(down, 2), "total": round(up + down, 2)},
            "link_gb_s": round(frames * (up + down) / el / 1e9, 2)}


VERIFY_COLUMNS = ("status", "ip_csum", "l4_csum")


def e2e_rate(sh, device, chunks=16, reps=3, columns=None, verify=None, seconds=1.5, priorities=True, depth=4):
    """PCIe-inclusive rate: pinned host frames -> H2D -> kernel -> D2H of the results,
    on two alternating streams with `depth` buffer sets, paced as a producer is:
    a buffer set is reused once its previous chunk is back (at most `depth`
    chunks in flight; 4, the ring's slot count, moved 76-80 GB/s of link
    traffic where 2 moved 55-68 and 3 62 on one box,
    profiles/r06/e2e/ring_factor_probe_depth.txt), the second stream starts one
    upload behind the first, and the two streams have different priorities, so
    HIP never puts them on one hardware queue (which serializes every copy:
    ~54 GB/s instead of 70-79, profiles/r06/e2e/hwq_probe*.txt); enqueueing
    every chunk up front moved 53-57 (tools/ring_factor_probe.py). Fixed-stride batches ship the frames only;
    descriptor batches (IMIX) ship each chunk's frame span plus its compact
    descriptors (u32 offset rebased to the chunk + u16 length, 6 B/frame) with
    the size hint the ring would give. Reported beside `value`, never as `value`.
    `stages`: per-stage device time summed over the timed chunks (HIP events on
    the two streams, so H2D of one chunk overlaps the kernel / D2H of the other).
    verify(first_frame, n, result): called (tests) for the last two chunks after
    the timed region, with the device result they left in the two buffers."""
    columns = columns or lp.IPV4_COLUMNS
    w = sh.w
    n = sh.n
    per = n // chunks
    # two priorities: HIP draws hardware queues per priority, so the two streams
    # never share one (sharing serializes every copy; as the ring, ring.cpp)
    lo_prio, hi_prio = torch.cuda.Stream.priority_range() if priorities else (0, 0)
    streams = [torch.cuda.Stream(device, priority=lo_prio), torch.cuda.Stream(device, priority=hi_prio)]
    res = [lp.RxResult(per, device, columns, counters=False) for _ in range(depth)]
    hout = [torch.empty(r.nbytes, dtype=torch.uint8).pin_memory() for r in res]
    if w.stride:
        stride = w.stride
        host = torch.from_numpy(w.buf[: n * stride]).pin_memory()
        spans = [(k * per * stride, (k + 1) * per * stride) for k in range(chunks)]
        desc = None
        up_desc = 0
    else:
        offs, lens = w.offsets[: per * chunks], w.lengths[: per * chunks]
        if int(lens.max()) > 0xFFFF:
            return None
        spans = [(int(offs[k * per]), int(offs[(k + 1) * per - 1] + lens[(k + 1) * per - 1])) for k in range(chunks)]
        if max(e - b for b, e in spans) > 0xFFFFFFFF:
            return None
        host = torch.from_numpy(w.buf[: spans[-1][1]]).pin_memory()
        rebased = np.concatenate([(offs[k * per:(k + 1) * per] - np.uint64(spans[k][0])).astype(np.uint32)
                                  for k in range(chunks)])
        h_off = torch.from_numpy(rebased.view(np.int32)).pin_memory()
        h_len = torch.from_numpy(lens.astype(np.uint16).view(np.int16)).pin_memory()
        d_off = [torch.empty(per, dtype=torch.int32, device=device) for _ in range(depth)]
        d_len = [torch.empty(per, dtype=torch.int16, device=device) for _ in range(depth)]
        hints = [lp.desc_size_hint(lens[k * per:(k + 1) * per]) for k in range(chunks)]
        desc = (h_off, h_len, d_off, d_len, hints)
        up_desc = 6
    span_max = max(e - b for b, e in spans)
    dbuf = [torch.empty(span_max + 32, dtype=torch.uint8, device=device) for _ in range(depth)]
    for d in dbuf:
        d.zero_()                                     # the granule tail past every span reads zeros
    ev = {}

    done = [None] * depth
    up = [None] * depth
    seq = [0]                                  # chunks issued: buffer set seq % depth, stream seq % 2
    last = {}                                  # chunk -> the buffer set that holds its last result

    def chunk(k, timed):
        s, j = streams[seq[0] % 2], seq[0] % depth
        seq[0] += 1
        last[k] = j
        b, e = spans[k]
        if done[j] is not None:
            done[j].synchronize()        # a producer reuses a buffer pair once its last chunk is back
        with torch.cuda.stream(s):
            if timed:
                marks = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
                marks[0].record(s)
            dbuf[j][: e - b].copy_(host[b:e], non_blocking=True)
            up[j] = torch.cuda.Event()
            up[j].record(s)
            if desc is None:
                if timed:
                    marks[1].record(s)
                lp.rx_process(dbuf[j], stride=w.stride, frame_len=w.stride, n_frames=per, out=res[j], stream=s)
            else:
                h_off, h_len, d_off, d_len, hints = desc
                d_off[j].copy_(h_off[k * per:(k + 1) * per], non_blocking=True)
                d_len[j].copy_(h_len[k * per:(k + 1) * per], non_blocking=True)
                if timed:
                    marks[1].record(s)
                lp.rx_process(dbuf[j], offsets=d_off[j], lengths=d_len[j], out=res[j], stream=s,
                              flags=lp.DESC_COMPACT | hints[k])
            if timed:
                marks[2].record(s)
            res[j].to_host(hout[j], stream=s)             # every record column in one D2H
            if timed:
                marks[3].record(s)
                ev.setdefault("marks", []).append(marks)
            done[j] = torch.cuda.Event()
            done[j].record(s)

    # one untimed pass over the batch first: the first pass from a freshly
    # pinned buffer measured ~60 % of the later ones (profiles/r05/ring/); a
    # second one sizes the timed region to about `seconds` (at least `reps`
    # passes), comparable with the ring lines' few seconds
    for k in range(chunks):
        chunk(k, False)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    for k in range(chunks):
        chunk(k, False)
    torch.cuda.synchronize()
    reps = max(reps, int(seconds / max(time.perf_counter() - t1, 1e-4)))
    t0 = time.perf_counter()
    for r in range(reps):
        for k in range(chunks):
            chunk(k, True)
            if r == 0 and k == 0:
                up[last[0]].synchronize()    # stagger: stream 1 starts once stream 0's first upload is done
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    if verify:
        for k in (chunks - 2, chunks - 1):
            verify(k * per, per, res[last[k]])
    frames = reps * chunks * per
    nbytes = reps * sum(e - b for b, e in spans)
    st = {"h2d_s": 0.0, "kernel_s": 0.0, "d2h_s": 0.0}
    for m in ev.get("marks", []):
        st["h2d_s"] += m[0].elapsed_time(m[1]) / 1e3
        st["kernel_s"] += m[1].elapsed_time(m[2]) / 1e3
        st["d2h_s"] += m[2].elapsed_time(m[3]) / 1e3
    rb = lp.engine.column_bytes(columns)
    return {"mpkts_s": round(frames / el / 1e6, 1), "gb_s": round(nbytes / el / 1e9, 2),
            **_link(frames, el, nbytes / frames + up_desc, res[0].nbytes / per),
            "stages": {"wall_s": round(el, 4), **{k: round(v, 4) for k, v in st.items()},
                       "h2d_gb_s": round(nbytes / st["h2d_s"] / 1e9, 2) if st["h2d_s"] else None,
                       "host_threads": 1},
            "note": "pinned host batch -> hipMemcpyAsync H2D -> rx kernel -> one D2H of the packed record "
                    f"columns ({rb} B/frame: {', '.join(columns)}), {chunks} chunks on 2 streams of different priorities "
                    f"with {depth} buffer sets, at most {depth} in flight, the second stream started one upload "
                    "behind the first"
                    + ("" if desc is None else "; descriptor batch: each chunk's frame span + compact descriptors "
                                               "(6 B/frame) up, with the size hint pnetgpu_desc_size_hint gives")}


def _ring_link(frames, nbytes, el, rb, nbatches, desc_bytes):
    # up: the frames plus the descriptors the ring shipped (none for batches of
    # uniform frames, which go as fixed-stride batches; compact, 6 B a frame,
    # otherwise: pnetgpu_ring_stats.desc_bytes); down: the record columns plus
    # 64 B of counters per batch
    return _link(frames, el, (nbytes + desc_bytes) / frames, rb + 64 * nbatches / frames)


def _ring_stages(ring, el):
    """Where a ring line's wall time went (pnetgpu_ring_stats): host seconds in
    push_many (descriptors + copies), submit (enqueueing) and wait (blocked on
    the oldest batch), the rest of the host loop, and the device stage sums."""
    st = ring.stats()
    host = {k: st[k + "_ns"] / 1e9 for k in ("push", "submit", "wait")}
    out = {"wall_s": round(el, 4), **{f"{k}_s": round(v, 4) for k, v in host.items()},
           "other_host_s": round(el - sum(host.values()), 4),
           "h2d_s": round(st["h2d_ms"] / 1e3, 4), "kernel_s": round(st["kernel_ms"] / 1e3, 4),
           "d2h_s": round(st["d2h_ms"] / 1e3, 4), "batches": st["batches"], "timed_batches": st["timed_batches"],
           "stride_batches": st["stride_batches"], "desc_bytes": st["desc_bytes"], "host_threads": st["host_threads"]}
    if st["push_ns"]:
        out["push_gb_s"] = round(st["bytes"] / (st["push_ns"] / 1e9) / 1e9, 2)
    if st["h2d_ms"]:
        out["h2d_gb_s"] = round(st["bytes"] / (st["h2d_ms"] / 1e3) / 1e9, 2)
    return out


def _ring_warm(ring, feed):
    """One untimed pass of the producer over its source, then zeroed statistics:
    a ring's first batches run slow (first DMA from freshly pinned or registered
    pages; the plain pipeline's e2e_rate has the same untimed pass)."""
    for b in feed():
        del b
    for b in ring.drain():
        del b
    ring.reset_stats()


def _ring_source(sh):
    w = sh.w
    n = min(sh.n, 1 << 22)
    if w.stride:
        offs = np.arange(n, dtype=np.uint64) * np.uint64(w.stride)
        lens = np.full(n, w.frame_len, dtype=np.uint32)
    else:
        offs, lens = w.offsets[:n], w.lengths[:n]
    return offs, lens


def e2e_ring_rate(sh, seconds=3.0, columns=None, slots=None, stage_times=True):
    """Producer-inclusive rate: frames copied into the pinned ring
    (pnetgpu_ring_push_many: the DataLinkReceiver::next() consumer), shipped,
    verified and the record columns copied back (rotating slots: one filling,
    one held by the consumer, the rest in flight)."""
    columns = columns or lp.IPV4_COLUMNS
    w = sh.w
    offs, lens = _ring_source(sh)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False, columns=columns, slots=slots,
                   stage_times=stage_times)
    nslots = ring.slots
    _ring_warm(ring, lambda: ring.feed_many(w.buf, offs, lens))
    frames = nbytes = nb = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        for b in ring.feed_many(w.buf, offs, lens):
            frames += b.n
            nbytes += b.counters["bytes"]          # the GPU counted them
            nb += 1
            del b
    for b in ring.drain():
        frames += b.n
        nbytes += b.counters["bytes"]          # the GPU counted them
        nb += 1
    el = time.perf_counter() - t0
    stages = _ring_stages(ring, el)
    ring.close()
    rb = lp.engine.column_bytes(columns)
    return {"mpkts_s": round(frames / el / 1e6, 1), "gb_s": round(nbytes / el / 1e9, 2),
            **_ring_link(frames, nbytes, el, rb, nb, stages["desc_bytes"]), "stages": stages,
            "note": "host frames pushed into the pinned ring with pnetgpu_ring_push_many (descriptors and "
                    f"non-temporal frame copies on a persistent pool of {stages['host_threads']} host threads), "
                    f"async H2D -> rx kernel -> D2H of the record columns ({rb} B/frame: {', '.join(columns)}), "
                    f"{nslots} rotating slots of 64 MiB / 1 Mi frames on 2 alternating streams; batches of "
                    "uniform frames at a constant stride ship as fixed-stride batches, without descriptors "
                    "(stages.stride_batches)",
            "slots": nslots}


def e2e_zero_copy_rate(sh, seconds=3.0, columns=None, slots=None, stage_times=True):
    """Zero-copy producer: the host frames stay where they are (a registered
    buffer, as an mmap'd pcap file or AF_PACKET ring would be) and each batch is
    one DMA of their span (pnetgpu_ring_submit_region), verified, and every
    record column copied back (rotating slots)."""
    columns = columns or lp.IPV4_COLUMNS
    w = sh.w
    offs, lens = _ring_source(sh)
    span = int(offs[-1] + lens[-1])
    buf = w.buf[:span]
    reg = lp.HostRegistration(buf)
    ring = lp.Ring(batch_bytes=64 << 20, batch_frames=1 << 20, copy=False, columns=columns, slots=slots,
                   stage_times=stage_times)
    nslots = ring.slots
    frames = nbytes = nb = 0
    try:
        _ring_warm(ring, lambda: ring.feed_region(buf, offs, lens))
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < seconds:
            for b in ring.feed_region(buf, offs, lens):
                frames += b.n
                nbytes += b.counters["bytes"]          # the GPU counted them
                nb += 1
                del b
        for b in ring.drain():
            frames += b.n
            nbytes += b.counters["bytes"]          # the GPU counted them
            nb += 1
        el = time.perf_counter() - t0
        stages = _ring_stages(ring, el)
    finally:
        ring.close()
        reg.close()
    rb = lp.engine.column_bytes(columns)
    return {"mpkts_s": round(frames / el / 1e6, 1), "gb_s": round(nbytes / el / 1e9, 2),
            **_ring_link(frames, nbytes, el, rb, nb, stages["desc_bytes"]), "stages": stages,
            "note": "frames DMA'd straight from a registered host buffer (pnetgpu_ring_submit_region, no copy into "
                    f"the ring), rx kernel, D2H of the record columns ({rb} B/frame: {', '.join(columns)}; "
                    f"pnetgpu_ring_set_columns), {nslots} rotating slots of 64 MiB / 1 Mi frames on 2 alternating streams; "
                    "batches of uniform frames at a constant stride ship as fixed-stride batches, without descriptors "
                    "(stages.stride_batches)",
            "slots": nslots}


def pack_rate(sh, seconds=1.0):
    """The ring producer's host ceiling on its own: pnetgpu_batch_pack of the same
    frames into a 64-MiB pinned batch (the push_many pass, no GPU work)."""
    offs, lens = _ring_source(sh)
    dst = torch.empty(64 << 20, dtype=torch.uint8).pin_memory().numpy()
    do = np.empty(len(offs), np.uint64)
    dl = np.empty(len(offs), np.uint32)
    frames = nbytes = 0
    i = 0
    lp.batch_pack(sh.w.buf, offs[:1 << 16], lens[:1 << 16], dst, do, dl)     # the pool starts
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        k, b = lp.batch_pack(sh.w.buf, offs[i:i + (1 << 20)], lens[i:i + (1 << 20)], dst, do, dl, check_bounds=False)
        frames += k
        nbytes += b
        i = (i + k) % len(offs)
    el = time.perf_counter() - t0
    return {"gb_s": round(nbytes / el / 1e9, 2), "mpkts_s": round(frames / el / 1e6, 1),
            "host_threads": lp.host_threads(),
            "note": "pnetgpu_batch_pack into one 64-MiB pinned batch (descriptors + non-temporal copies), host only"}


def time_launches(fn, steps, warmup, stream):
    """Average duration (ms) of `steps` back-to-back launches of fn(stream): one HIP
    event pair on that stream around all of them (see time_shard)."""
    for _ in range(warmup):
        fn(stream)
    stream.synchronize()
    a = torch.cuda.Event(enable_timing=True)
    b = torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for _ in range(steps):
        fn(stream)
    b.record(stream)
    stream.synchronize()
    return a.elapsed_time(b) / steps


def tx_sector_writes(sh):
    """Bytes the HBM must write per launch to patch the two checksum fields in
    place: every 32-B sector that holds a byte of either field (the IPv4 header
    checksum at frame offset 24, the L4 checksum at 34 + 6 / 16 / 2 for UDP /
    TCP / ICMP), counted per frame from the frame offsets; the status column
    adds 2 B per frame. For 64-B frames the two fields sit in the frame's two
    sectors, so the floor is the whole frame (rs_sender.rs:38-39,70-71 patch
    both)."""
    w = sh.w
    offs = np.arange(sh.n, dtype=np.int64) * w.stride
    proto = sh.w.buf[offs[:1] + 23][0] if sh.n else 17
    l4 = 34 + {17: 6, 6: 16, 1: 2}.get(int(proto), 6)
    sec = np.stack([(offs + p) // 32 for p in (24, 25, l4, l4 + 1)], axis=1)
    sec.sort(axis=1)
    distinct = 1 + (np.diff(sec, axis=1) != 0).sum(axis=1)
    return int(distinct.sum()) * 32 + 2 * sh.n


def tx_fill_rate(sh, steps, warmup, device):
    """Sender side (configs[0] builds and checksums frames
    the way benches/rs_sender.rs:38-39,70-71 does): pnetgpu_tx_fill_checksums over
    a device copy of the batch, every IPv4 header and L4 checksum written in place,
    plus the status column. Beside it, the oracle's scalar oracle_tx_fill on one
    core over the first 2^20 frames."""
    from oracle import coracle  # CPU baseline only
    w = sh.w
    if not w.stride:
        return None
    small = w.frame_len <= 64
    data = sh.data.clone()
    res = lp.RxResult(sh.n, device, ("status",), counters=False)
    stream = torch.cuda.Stream(device)
    ms = time_launches(lambda s: lp.tx_fill_checksums(data, stride=w.stride, frame_len=w.frame_len, n_frames=sh.n,
                                                      out=res, stream=s), steps, warmup, stream)
    kernel = lp.last_rx_kernel()
    alg = sh.frame_bytes + sh.n * (4 + 2)   # frames read, two checksum fields + status written
    n1 = min(sh.n, 1 << 20)
    t0 = time.perf_counter()
    coracle.tx_fill(w.buf[: n1 * w.stride], n1, stride=w.stride, frame_len=w.frame_len)
    cpu = n1 / (time.perf_counter() - t0) / 1e6
    del data
    out = {"workload": sh.name, "kernel": kernel, "mpkts_s": round(sh.n / (ms * 1e-3) / 1e6, 1),
           "kernel_avg_ms": round(ms, 4),
           "alg_bytes_per_launch": alg,
           "achieved_gbs": round(alg / (ms * 1e-3) / 1e9, 1), "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
           "cpu_port_1core_mpkts_s": round(cpu, 2), "traffic": load_traffic(f"tx_{sh.name}"),
           "note": "device-resident tx_fill_checksums (IPv4 header + L4 checksum patched in place), kernel time; "
                   f"CPU: oracle_tx_fill, 1 core, first {n1} frames"}
    # what the writes cost in HBM: PMC WRITE_SIZE per frame against the 4 B of
    # checksum fields that change (profiles/pmc_tx_<workload>.json; the sector
    # floor of two fields in two 32-B sectors is 64 B: profiles/r04/tx_writes/)
    # the same kernel time against the sector floor: frames read once plus
    # every 32-B sector holding a checksum byte written (what a patch in place
    # must write; `frac` counts only the 4 changed bytes per frame)
    floor = sh.frame_bytes + tx_sector_writes(sh)
    out["sector_floor_bytes_per_launch"] = floor
    out["frac_sector_floor"] = round(floor / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
    wb = load_traffic(f"tx_{sh.name}", "write_bytes_per_launch")
    if wb:
        out["pmc_write_bytes_per_frame"] = round(wb / sh.n, 1)
        out["write_over_alg_writes"] = round(wb / (sh.n * 4), 2)
    if small:
        # the small kernel writes every patched frame back whole (coalesced 1-KiB stores:
        # 2-B patches at scattered offsets ran 1.7x slower), so it moves ~2x the frame bytes
        out["rewrite_gbs"] = round((2 * sh.frame_bytes + 2 * sh.n) / (ms * 1e-3) / 1e9, 1)
    else:
        # the MTU kernel stores the two 2-B checksum fields only (byte stores into the
        # frame's first line); the traffic key says what HBM saw
        out["store"] = "2 x 2-B field stores per frame"
        # the alternative to patching in place: the same checksums as a
        # 4-B-per-frame column pair (rx_process with ip_csum + l4_csum only), for a
        # consumer whose H2D / NIC path patches the two words itself
        cols = lp.RxResult(sh.n, device, ("ip_csum", "l4_csum"), counters=False)
        ms_c = time_launches(lambda s: lp.rx_process(sh.data, stride=w.stride, frame_len=w.frame_len, n_frames=sh.n,
                                                     out=cols, stream=s), steps, warmup, stream)
        alg_c = sh.frame_bytes + sh.n * 4
        out["checksum_columns_instead"] = {
            "kernel_avg_ms": round(ms_c, 4), "mpkts_s": round(sh.n / (ms_c * 1e-3) / 1e6, 1),
            "alg_bytes_per_launch": alg_c, "frac": round(alg_c / (ms_c * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": "rx_process writing only the ip_csum and l4_csum columns (4 B/frame, coalesced) instead of "
                    "patching the frames in place"}
    return out


def descriptor_rate(sh, steps, warmup, device):
    """The same fixed-size frames handed over as a descriptor batch (compact
    descriptors, as the ring and the AF_PACKET path ship them): kernel time with
    no size hint (the mixed shape, which streams runs of large or jumbo frames
    in the MTU / jumbo order itself) and with the hint pnetgpu_desc_size_hint
    gives for their lengths (DESC_HINT_LARGE -> the MTU shape, DESC_HINT_JUMBO
    -> the jumbo shape). Algorithmic
    bytes = frames + 26-B record + 6-B descriptor per frame."""
    w = sh.w
    if not w.stride or w.buf is None:
        return None
    n = sh.n
    if n * w.stride > 0xFFFFFFFF or w.frame_len > 0xFFFF:
        return None                                     # compact descriptors cannot describe it
    # u32 offsets held in an int32 tensor (the kernel reads them unsigned)
    offs = torch.from_numpy((np.arange(n, dtype=np.uint64) * np.uint64(w.stride)).astype(np.uint32).view(np.int32))
    offs = offs.to(device)
    lens = torch.full((n,), w.frame_len, dtype=torch.int16, device=device)
    hint = lp.desc_size_hint(np.full(n, w.frame_len, np.uint32))
    res = lp.RxResult(n, device, lp.IPV4_COLUMNS, counters=False)
    stream = torch.cuda.Stream(device)
    alg = sh.frame_bytes + n * (26 + 6)
    out = {"hint_flag": {0: "none", lp.DESC_HINT_LARGE: "DESC_HINT_LARGE", lp.DESC_HINT_JUMBO: "DESC_HINT_JUMBO"}[hint]}
    for label, fl in (("no_hint", 0), ("with_hint", hint)):
        ms = time_launches(lambda s: lp.rx_process(sh.data, offsets=offs, lengths=lens, out=res, stream=s,
                                                   flags=lp.DESC_COMPACT | fl), steps, warmup, stream)
        out[label] = {"kernel": lp.last_rx_kernel(), "kernel_avg_ms": round(ms, 4),
                      "mpkts_s": round(n / (ms * 1e-3) / 1e6, 1),
                      "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)}
    out["note"] = (f"{n} frames of {w.frame_len} B as a compact-descriptor batch; alg bytes = frames + 32 B/frame "
                   "(26-B record + 6-B descriptor)")
    return out


def slices_rate(sh, steps, warmup, device):
    """Batched util::ipv4_checksum (pnetgpu_ipv4_checksum_slices, the
    tcp::ipv4_checksum call of tcp.rs:239-248) over every TCP segment of the
    1500-B batch: slice = frame[34, 1500), skipword 8, the frame's own addresses."""
    w = sh.w
    if not w.stride or sh.name != "tcp1500":
        return None
    n = sh.n
    base = np.arange(n, dtype=np.int64) * w.stride
    offs = torch.from_numpy(base + 34).to(device)
    lens = torch.full((n,), w.frame_len - 34, dtype=torch.int32, device=device)
    skips = torch.full((n,), 8, dtype=torch.int32, device=device)
    frames = w.buf[: n * w.stride].reshape(n, w.stride)
    addrs = torch.from_numpy(np.ascontiguousarray(frames[:, 26:34])).to(device)
    protos = torch.full((n,), 6, dtype=torch.uint8, device=device)
    stream = torch.cuda.Stream(device)
    ms = time_launches(lambda s: lp.ipv4_checksum_slices(sh.data, offs, lens, skips, addrs, protos, stream=s),
                       steps, warmup, stream)
    alg = n * (w.frame_len - 34 + 8 + 12 + 4 + 1 + 2)   # slice + addrs + descriptor + skipword + proto + result
    return {"mslices_s": round(n / (ms * 1e-3) / 1e6, 1), "kernel_avg_ms": round(ms, 4),
            "achieved_gbs": round(alg / (ms * 1e-3) / 1e9, 1), "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
            "note": f"{n} TCP segments of {w.frame_len - 34} B, util::ipv4_checksum per slice, kernel time"}


CAPTURED_TCP_FRAME = bytes.fromhex(   # pnet_packet/benches/packet_benchmarks.rs:63 (bench_ipv4_parsing)
    "000c291ce319ecf4bbd93e7d08004500002e1b6540008006cd76c0a8c887c0a8c8151a3707d0dd6abb2b1f5fd25150180402120f"
    "000068656c6c6f0a")


def refshapes_block(steps, warmup, device):
    """The reference's own micro-benchmark shapes, batched on the GPU with the
    oracle's CPU rate beside them:
      checksum_small  util::checksum(&[99u8; 20], 5)    checksum_benchmarks.rs:8-12
      checksum_large  util::checksum(&[123u8; 1024], 5) checksum_benchmarks.rs:14-18
      ipv4_parsing    the captured 60-B TCP frame through the receive chain
                      (Ipv4Packet::new over its Ethernet payload, then the rest
                      of packetdump's chain), packet_benchmarks.rs:63-71
    Slices are packed back to back, one (u64 offset, u32 length, u32 skipword)
    descriptor each; algorithmic bytes = slice bytes + 16 B descriptor + 2 B result.
    `compact`: the same slices through pnetgpu_checksum_slices_compact (8-B
    pnetgpu_slice_desc records; algorithmic bytes = slice + 8 B + 2 B result).
    `strided`: the same slices through pnetgpu_checksum_slices_strided (no
    descriptor arrays; algorithmic bytes = slice + 2 B result)."""
    from oracle import coracle  # CPU baseline legs only
    out = {}
    stream = torch.cuda.Stream(device)
    for name, fill, size, n in (("checksum_small", 99, 20, 1 << 24), ("checksum_large", 123, 1024, 1 << 20)):
        buf = np.full(n * size + 32, fill, dtype=np.uint8)
        offs = np.arange(n, dtype=np.uint64) * np.uint64(size)
        lens = np.full(n, size, dtype=np.uint32)
        skips = np.full(n, 5, dtype=np.uint32)
        d = torch.from_numpy(buf).to(device)
        do, dl, ds = (torch.from_numpy(offs.view(np.int64)).to(device), torch.from_numpy(lens.view(np.int32)).to(device),
                      torch.from_numpy(skips.view(np.int32)).to(device))
        res = {}
        ms = time_launches(lambda s: res.__setitem__("o", lp.checksum_slices(d, do, dl, ds, stream=s)), steps, warmup,
                           stream)
        kern = lp.last_rx_kernel()
        got = res["o"].cpu().numpy().view(np.uint16)
        want = coracle.checksum(bytes([fill] * size), 5)
        alg = n * (size + 16 + 2)
        cpu_out = np.zeros(n, np.uint16)
        k = min(n, 1 << 20)
        cpu = {}
        for label, nt in (("1core", 1), ("all", usable_cpus())):
            reps, el = _timed_reps(lambda r: coracle.checksum_slices_reps(buf, offs[:k], lens[:k], skips[:k],
                                                                          cpu_out[:k], nthreads=nt, reps=r), 1.0)
            cpu[label] = round(k * reps / el / 1e6, 1)
        # the same slices through 8-B compact descriptors (pnetgpu_checksum_slices_compact)
        dc = lp.slice_descriptors(offs, lens, skips, device=device)
        ms_c = time_launches(lambda s: res.__setitem__("c", lp.checksum_slices_compact(d, dc, stream=s)),
                             steps, warmup, stream)
        kern_c = lp.last_rx_kernel()
        got_c = res["c"].cpu().numpy().view(np.uint16)
        alg_c = n * (size + 8 + 2)
        compact = {"kernel_avg_ms": round(ms_c, 4), "mslices_s": round(n / (ms_c * 1e-3) / 1e6, 1),
                   "achieved_gbs": round(alg_c / (ms_c * 1e-3) / 1e9, 1),
                   "frac": round(alg_c / (ms_c * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "parity": bool((got_c == want).all()), "alg_bytes_per_slice": size + 8 + 2, "kernel": kern_c}
        del dc
        # the same slices without descriptor arrays (pnetgpu_checksum_slices_strided)
        ms_st = time_launches(lambda s: res.__setitem__("s", lp.checksum_slices_strided(d, n, size, size, 5, stream=s)),
                              steps, warmup, stream)
        kern_st = lp.last_rx_kernel()
        got_st = res["s"].cpu().numpy().view(np.uint16)
        alg_st = n * (size + 2)
        strided = {"kernel_avg_ms": round(ms_st, 4), "mslices_s": round(n / (ms_st * 1e-3) / 1e6, 1),
                   "achieved_gbs": round(alg_st / (ms_st * 1e-3) / 1e9, 1),
                   "frac": round(alg_st / (ms_st * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                   "parity": bool((got_st == want).all()), "alg_bytes_per_slice": size + 2, "kernel": kern_st}
        out[name] = {"slices": n, "slice_bytes": size, "skipword": 5, "kernel": kern, "kernel_avg_ms": round(ms, 4),
                     "mslices_s": round(n / (ms * 1e-3) / 1e6, 1),
                     "achieved_gbs": round(alg / (ms * 1e-3) / 1e9, 1),
                     "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                     "parity": bool((got == want).all()), "expected": int(want),
                     "cpu_port_1core_mslices_s": cpu["1core"], "cpu_port_all_mslices_s": cpu["all"],
                     "compact": compact, "strided": strided}
        del d, do, dl, ds
    # ipv4_parsing: the captured frame replicated at a 64-B stride (the small kernel)
    n = 1 << 24
    frame = np.frombuffer(CAPTURED_TCP_FRAME + bytes(64 - len(CAPTURED_TCP_FRAME)), np.uint8)
    buf = np.concatenate([np.tile(frame, n), np.zeros(32, np.uint8)])
    d = torch.from_numpy(buf).to(device)
    res = lp.RxResult(n, device, lp.IPV4_COLUMNS, counters=True)
    flen = len(CAPTURED_TCP_FRAME)
    ms = time_launches(lambda s: lp.rx_process(d, stride=64, frame_len=flen, n_frames=n, out=res, stream=s), steps,
                       warmup, stream)
    rec = coracle.rx_frame(CAPTURED_TCP_FRAME)
    got = res.numpy()
    parity = all(bool((got[c] == rec[c]).all()) for c in lp.IPV4_COLUMNS)
    alg = n * (flen + lp.column_bytes(lp.IPV4_COLUMNS))
    recs = np.zeros(1 << 20, dtype=coracle.REC_DTYPE)
    cpu = {}
    for label, nt in (("1core", 1), ("all", usable_cpus())):
        reps, el = _timed_reps(lambda r: coracle.rx_batch_reps(buf, 1 << 20, stride=64, frame_len=flen, nthreads=nt,
                                                               reps=r, out=recs), 1.0)
        cpu[label] = round((1 << 20) * reps / el / 1e6, 1)
    out["ipv4_parsing"] = {"frames": n, "frame_bytes": flen, "stride": 64, "kernel_avg_ms": round(ms, 4),
                           "mpkts_s": round(n / (ms * 1e-3) / 1e6, 1),
                           "achieved_gbs": round(alg / (ms * 1e-3) / 1e9, 1),
                           "frac": round(alg / (ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4), "parity": parity,
                           "cpu_port_1core_mpkts_s": cpu["1core"], "cpu_port_all_mpkts_s": cpu["all"]}
    out["note"] = ("GPU kernel time over device-resident batches (IPv4 record columns for ipv4_parsing); frac "
                   "= algorithmic bytes (slice or frame + descriptor + result) / kernel time / 8 TB/s; CPU: the "
                   "oracle's scalar restatement over the first 2^20 items")
    return out


def load_traffic(workload, key="hbm_bytes_per_launch"):
    """HBM bytes per launch from the committed rocprofv3 PMC summary (profiles/), if present."""
    p = os.path.join(ROOT, "profiles", f"pmc_{workload}.json")
    if not os.path.exists(p):
        return None
    try:
        with open(p) as fh:
            d = json.load(fh)
        return d.get(key)
    except Exception:
        return None


def load_library():
    """Import the HIP library's binding (ranks only; also used by tools/ that reuse Shard)."""
    global lp, shard
    import libpnet_amd as _lp
    from libpnet_amd import shard as _shard
    lp, shard = _lp, _shard
    return _lp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(n):
    """`python bench.py --gpus N` (N > 1, no WORLD_SIZE in the environment): start
    the N ranks with torchrun as a CHILD process (one process per GPU, RANK /
    LOCAL_RANK / WORLD_SIZE from torchrun) and exit with its status. This parent
    never touches the GPU and never execs (the children initialise the GPUs)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    log(f"[bench] --gpus {n}: starting {n} ranks: {' '.join(cmd)}")
    return subprocess.run(cmd, env=env).returncode


def launch_check(args, world, rank):
    """--launch-check: the multi-rank harness without the GPU (CPU test of the
    driver's `bench.py --gpus N` shape, gloo). Each rank takes its byte-balanced
    shard of a small IMIX length vector (shard.shard_by_bytes, the configs[3]
    partition), the counters are all-reduced and the time max-reduced exactly as
    in a GPU run, and rank 0 prints the line."""
    import libpnet_amd.shard as shard_mod
    rng = np.random.default_rng(args.seed)
    n = 100003
    lengths = rng.choice(np.array([64, 576, 1500], dtype=np.uint32), size=n, p=[7 / 12, 4 / 12, 1 / 12])
    t0 = time.perf_counter()
    # as in a GPU run: rank 0 cuts the global vector, every rank receives the cuts
    lo, hi = shard_mod.broadcast_byte_cuts(lambda: lengths, world, rank)
    assert (lo, hi) == shard_mod.shard_by_bytes(lengths, world, rank)
    ctr = torch.tensor([hi - lo, int(lengths[lo:hi].sum()), rank], dtype=torch.int64)
    shard_mod.all_reduce_counters(ctr)
    wall = shard_mod.all_reduce_max(time.perf_counter() - t0, "cpu")
    bmin, bmax = shard_mod.all_reduce_min_max(float(lengths[lo:hi].sum()), "cpu")
    ok = int(ctr[0]) == n and int(ctr[1]) == int(lengths.sum()) and int(ctr[2]) == world * (world - 1) // 2
    if rank == 0:
        coll = ({"backend": str(torch.distributed.get_backend()), "world_size": torch.distributed.get_world_size()}
                if torch.distributed.is_initialized() else {"backend": None, "world_size": 1})
        print(json.dumps({"metric": METRIC, "launch_check": True, "n_gpus": world, "world_size": world,
                          "collective": coll,
                          "frames": int(ctr[0]), "bytes": int(ctr[1]), "wall_s": wall, "counters_ok": ok,
                          "shard_bytes_min": int(bmin), "shard_bytes_max": int(bmax)}),
              flush=True)
    return 0 if ok else 1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks (one per GPU); without WORLD_SIZE set, N > 1 starts them with torchrun")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workloads", default="udp64,tcp1500,udp1500,imix,udp6_jumbo,udp64_verify,imix_verify",
                    help="first one is the headline `value`; the others are reported under `workloads`")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-extra", action="store_true", help="skip the TX-fill and checksum-slices rates")
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--launch-check", action="store_true",
                    help="rank start-up, shard_by_bytes partition and the reductions only (no GPU; gloo)")
    ap.add_argument("--frames-scale", type=float, default=1.0,
                    help="scale every workload's frame count (rehearsals only; the bench line records it)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args.gpus)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist_on = world > 1
    if world != args.gpus:
        raise SystemExit(f"bench: WORLD_SIZE={world} but --gpus {args.gpus}: one rank per GPU")
    if args.launch_check:
        if dist_on:
            torch.distributed.init_process_group("gloo")
            assert torch.distributed.get_world_size() == world
        rc = launch_check(args, world, rank)
        if dist_on:
            torch.distributed.destroy_process_group()
        return rc

    load_library()
    # one rank per GPU; the modulo only matters for a rehearsal with more ranks
    # than GPUs (PNETGPU_BENCH_BACKEND=gloo, e.g. 2 ranks on a 1-GPU box)
    local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if dist_on:
        import datetime
        backend = os.environ.get("PNETGPU_BENCH_BACKEND", "nccl")   # nccl = RCCL over xGMI
        torch.distributed.init_process_group(backend, timeout=datetime.timedelta(minutes=10))
        assert torch.distributed.get_world_size() == world

    collective = {"backend": None, "world_size": 1, "library": None}     # one process: no collective runs
    if dist_on:
        collective = {"backend": str(torch.distributed.get_backend()),
                      "world_size": torch.distributed.get_world_size(),
                      "library": "RCCL" if str(torch.distributed.get_backend()) == "nccl" and torch.version.hip
                      else str(torch.distributed.get_backend())}
    names = [w for w in args.workloads.split(",") if w]
    results = {}
    primary = names[0]
    for name in names:
        cfg = WORKLOADS[name]
        t = time.perf_counter()
        n = max(64, int(cfg["n"] * args.frames_scale))
        # one global batch of world x n frames (the same seed on every rank), each
        # rank building and processing its shard: by frame index for the
        # fixed-size workloads, byte-balanced (shard.shard_by_bytes) for IMIX
        # (the configs[3] partition); weak scaling: n per GPU
        gname = cfg.get("synth", name)
        if gname == "imix":
            # the global length vector lives on rank 0 only; the cuts are broadcast
            lo, hi = shard.broadcast_byte_cuts(lambda: lp.synth.lengths(gname, n * world, args.seed * 1000), world,
                                               rank, device if dist_on and torch.distributed.get_backend() == "nccl"
                                               else None)
            partition = "shard_by_bytes"
        else:
            lo, hi = shard.shard_by_index(n * world, world, rank)
            partition = "shard_by_index"
        sh = Shard(name, hi - lo, args.seed * 1000, device, first=lo)
        sh.partition = partition
        if dist_on:
            # the host copy only serves the N=1 extras (CPU baseline, PCIe lines);
            # with 8 ranks on a node it would hold ~50 GB of host memory for nothing
            sh.w.buf = None
        if rank == 0:
            log(f"[bench] {name}: built {sh.n} frames ({sh.frame_bytes / 2**30:.2f} GiB) in {time.perf_counter() - t:.1f}s")
        ok, ctr = check_counters(sh)
        sh.kernel = lp.last_rx_kernel()      # the instantiation the launches use (rocprofv3's name)
        stream = torch.cuda.Stream(device)
        wall, avg_ms = time_shard(sh, args.steps, args.warmup, stream, dist_on)
        # counters: one RCCL all-reduce at the end (the "final throughput reduction")
        ctr_t = torch.tensor([ctr[k] for k in lp.COUNTER_NAMES] + [int(ok)], dtype=torch.int64, device=device)
        shard.all_reduce_counters(ctr_t)
        wall = shard.all_reduce_max(wall, device)
        n_all = torch.tensor([sh.n], dtype=torch.int64, device=device)
        shard.all_reduce_counters(n_all)              # frames of the whole batch (the shards' sum)
        frames_all = int(n_all.item()) * args.steps
        achieved = sh.alg_bytes / (avg_ms * 1e-3) / 1e9
        # every rank's kernel time: the spread shows shard imbalance (byte-balanced IMIX cuts)
        kmin, kmax = shard.all_reduce_min_max(avg_ms, device)
        results[name] = {
            "sh": sh, "wall": wall, "ms_per_step": wall / args.steps * 1e3,
            "mpkts_s": frames_all / wall / 1e6,
            "gb_s": int(ctr_t[lp.COUNTER_NAMES.index("bytes")].item()) * args.steps / wall / 1e9,
            "kernel_avg_ms": avg_ms, "kernel_ms_min": kmin, "kernel_ms_max": kmax,
            "frames_per_step": frames_all // args.steps,
            "achieved_gbs": achieved, "counters_ok": bool(ctr_t[-1].item() == world),
            "counters": {k: int(v) for k, v in zip(lp.COUNTER_NAMES, ctr_t[:-1].tolist())},
        }
        if rank == 0:
            r = results[name]
            log(f"[bench] {name}: {r['mpkts_s']:.1f} Mpkts/s, {r['gb_s']:.1f} GB/s frames, kernel avg "
                f"{avg_ms:.3f} ms -> {achieved:.0f} GB/s algorithmic ({achieved / HBM_PEAK_GBS:.1%} of 8 TB/s), "
                f"counters ok={r['counters_ok']}")

    if rank == 0:
        p = results[primary]
        sh = p["sh"]
        line = {
            "metric": METRIC,
            "value": round(p["mpkts_s"], 1),
            "unit": "Mpkts/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(p["ms_per_step"], 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (seeded splitmix64 frames, 1% with one flipped byte; built by libpnet_amd.synth)",
            "config": {
                "workload": WORKLOADS[primary]["desc"],
                "frames_per_gpu": sh.n,
                "frame_bytes": sh.w.frame_len,
                "batch_bytes_per_gpu": sh.frame_bytes,
                "mode": "fixed-stride" if sh.w.stride else "descriptor",
                "result_bytes_per_frame": sh.result_bytes,
                "parallelism": f"{getattr(sh, 'partition', 'shard_by_index')} x{world}",
                "global_batch_frames": results[primary]["frames_per_step"],
                **({"frames_scale": args.frames_scale} if args.frames_scale != 1.0 else {}),
            },
            "gb_s": round(p["gb_s"], 1),
            "roofline": {
                "bound": "hbm",
                "achieved": round(p["achieved_gbs"], 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(p["achieved_gbs"] / HBM_PEAK_GBS, 4),
                "traffic": load_traffic(primary),
                "traffic_source": f"profiles/pmc_{primary}.json: FETCH_SIZE/WRITE_SIZE from separate rocprofv3 --pmc "
                                  "passes over the same launch (tools/profile_round.sh), not measured in this run",
                "kernel": p["sh"].kernel,
                "kernel_avg_ms": round(p["kernel_avg_ms"], 4),
                "alg_bytes_per_launch": sh.alg_bytes,
            },
            "counters_ok": p["counters_ok"],
            # which collective library the reductions ran over, with how many
            # ranks it reported (null at N = 1: no process group)
            "collective": collective,
            "workloads": {},
        }
        for name, r in results.items():
            line["workloads"][name] = {
                "mpkts_s": round(r["mpkts_s"], 1), "gb_s": round(r["gb_s"], 1),
                "kernel_avg_ms": round(r["kernel_avg_ms"], 4),
                "kernel_ms_min": round(r["kernel_ms_min"], 4), "kernel_ms_max": round(r["kernel_ms_max"], 4),
                "frames_per_step": r["frames_per_step"],
                "roofline_frac": round(r["achieved_gbs"] / HBM_PEAK_GBS, 4),
                "achieved_gbs": round(r["achieved_gbs"], 1), "counters_ok": r["counters_ok"],
                "traffic": load_traffic(name), "kernel": r["sh"].kernel,
                "alg_bytes_per_launch": r["sh"].alg_bytes, "result_bytes_per_frame": r["sh"].result_bytes,
                "desc_bytes_per_frame": r["sh"].desc_bytes,
            }
        if world == 1 and not args.no_cpu:
            line["cpu_baseline"] = cpu_baseline(sh)
            for name, r in results.items():
                if name != primary and "synth" not in WORKLOADS[name]:   # not for a re-run of the same frames
                    line["workloads"][name]["cpu_baseline"] = cpu_baseline(r["sh"], target_s=1.5)
        if world == 1 and not args.no_extra:
            line["config0"] = config0_block(args.steps, args.warmup, device)
            line["reference_shapes"] = refshapes_block(args.steps, args.warmup, device)
            line["tx_fill"] = tx_fill_rate(sh, args.steps, args.warmup, device)
            for name in ("tcp1500", "udp1500"):
                if name in results and name != primary:
                    line["workloads"][name]["tx_fill"] = tx_fill_rate(results[name]["sh"], args.steps, args.warmup,
                                                                      device)
            for name in ("udp1500", "udp6_jumbo"):   # fixed-size frames as a descriptor batch, no hint / hint
                if name in results:
                    line["workloads"][name]["descriptor_mode"] = descriptor_rate(results[name]["sh"], args.steps,
                                                                               args.warmup, device)
            if "tcp1500" in results:
                line["workloads"]["tcp1500"]["ipv4_checksum_slices"] = slices_rate(results["tcp1500"]["sh"], args.steps,
                                                                                   args.warmup, device)
        if world == 1 and not args.no_e2e:
            # every e2e line ships the same 26-B IPv4 record, so they differ only
            # in the producer; the verify-only line (status + both checksums,
            # 6 B/frame back) shows the H2D-bound rate
            # the three producers of the same record, interleaved twice: the link's
            # rate drifts within a box, so each line keeps its better run and
            # lists both (runs_link_gb_s)
            runs = {"e2e_pcie": [], "e2e_zero_copy": [], "e2e_ring": []}
            for _ in range(2):
                runs["e2e_pcie"].append(e2e_rate(sh, device))
                runs["e2e_zero_copy"].append(e2e_zero_copy_rate(sh))
                runs["e2e_ring"].append(e2e_ring_rate(sh))
            for key, rs in runs.items():
                if rs[0] is None:
                    line[key] = None
                    continue
                best = dict(max(rs, key=lambda x: x["link_gb_s"]))
                best["runs_link_gb_s"] = [x["link_gb_s"] for x in rs]
                line[key] = best
            line["e2e_pcie_verify"] = e2e_rate(sh, device, columns=VERIFY_COLUMNS)
            line["e2e_pack_only"] = pack_rate(sh)
            # the 1500-B batches over the same pipeline (the link's large-frame rate)
            for name in ("udp1500", "tcp1500"):
                if name != primary and name in results and results[name]["sh"].w.buf is not None:
                    line["workloads"][name]["e2e_pcie"] = e2e_rate(results[name]["sh"], device)
                    if name == "udp1500":
                        line["workloads"][name]["e2e_zero_copy"] = e2e_zero_copy_rate(results[name]["sh"])
            # configs[3] (IMIX, compact descriptors up) and configs[4] (9000-B
            # jumbo frames, ~7,450 per 64-MiB ring batch) through all three producers
            for name in ("imix", "udp6_jumbo"):
                if name != primary and name in results and results[name]["sh"].w.buf is not None:
                    wsh = results[name]["sh"]
                    line["workloads"][name]["e2e_pcie"] = e2e_rate(wsh, device)
                    line["workloads"][name]["e2e_zero_copy"] = e2e_zero_copy_rate(wsh, seconds=2.0)
                    line["workloads"][name]["e2e_ring"] = e2e_ring_rate(wsh, seconds=2.0)
        print(json.dumps(line), flush=True)
    if dist_on:
        torch.distributed.barrier()
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main())
