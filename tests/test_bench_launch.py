"""The driver's multi-GPU command shape on CPU: `python bench.py --gpus N` with no
WORLD_SIZE must start N ranks itself (torchrun as a child process), each rank
must see world size N, the counters must all-reduce over the byte-balanced
shards and rank 0 alone must print one JSON line with n_gpus == N
(--launch-check: the harness without the GPU, gloo). The GPU twin with the HIP
kernel is tests/test_gpu_multi.py::test_bench_two_ranks_one_gpu."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None, timeout=240):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_lines(out):
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


@pytest.mark.parametrize("n", [1, 2, 3, 8])
def test_bench_gpus_n_starts_n_ranks(n):
    """N = 8 is the driver's scaling run: 8 ranks, byte cuts broadcast from rank 0."""
    p = _run(["--gpus", str(n), "--launch-check"])
    assert p.returncode == 0, p.stderr[-3000:]
    lines = _json_lines(p.stdout)
    assert len(lines) == 1, p.stdout          # rank 0 only
    line = lines[0]
    assert line["n_gpus"] == n and line["world_size"] == n
    # the line names the collective backend and the world size its process group reported
    if n == 1:
        assert line["collective"] == {"backend": None, "world_size": 1}       # one process: none ran
    else:
        assert line["collective"] == {"backend": "gloo", "world_size": n}
    assert line["counters_ok"] is True
    assert line["frames"] == 100003
    # byte-balanced: no rank's shard is more than one 1500-B frame off the mean
    mean = line["bytes"] / n
    assert line["shard_bytes_max"] - mean <= 1500 and mean - line["shard_bytes_min"] <= 1500


def test_bench_world_size_must_match_gpus():
    p = _run(["--gpus", "2", "--launch-check"], env_extra={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode != 0
    assert "one rank per GPU" in p.stderr
