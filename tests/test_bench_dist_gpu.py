"""bench.py's multi-rank path on the one GPU of a test box: two ranks (gloo for
the exchange, since RCCL refuses two ranks on one device), each holding half
of the rows, must return exactly the keys one rank holding all rows returns.
This runs the product's shard / all-gather / on-device merge code end to end
in separate processes (the driver's 8-GPU runs use the same code over RCCL)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _bench(tmp_path, tag, nproc, extra):
    out = str(tmp_path / f"{tag}.npy")
    args = ["bench.py", "--steps", "3", "--warmup", "1", "--no-cpu-baseline",
            "--no-secondary", "--dump-keys", out] + extra
    env = dict(os.environ, VS_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    if nproc > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
               f"--nproc-per-node={nproc}", "--master-addr", "127.0.0.1",
               "--master-port", str(_free_port())] + args
    else:
        cmd = [sys.executable] + args
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    line = [l for l in p.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line), np.load(out)


@pytest.mark.gpu
@pytest.mark.parametrize("config,rows", [("c3", 300_000), ("c3b1", 200_000)])
def test_two_ranks_equal_one_rank(tmp_path, config, rows):
    r1, k1 = _bench(tmp_path, f"{config}_one", 1, ["--config", config, "--rows", str(rows)])
    r2, k2 = _bench(tmp_path, f"{config}_two", 2, ["--config", config, "--rows", str(rows)])
    assert r2["n_gpus"] == 2 and r2["config"]["rows_per_gpu"] == rows // 2
    assert r1["config"]["rows_per_gpu"] == rows
    assert k1.shape == k2.shape and k1.shape[1] == 10
    np.testing.assert_array_equal(k1, k2)
    # each line prices ITS rank's launch, and carries HBM
    # traffic only when measured on exactly that many rows (none here)
    for r in (r1, r2):
        roof = r["roofline"]
        assert roof["bytes_per_launch"] >= r["config"]["rows_per_gpu"] * r["config"]["dim"]
        assert roof["bytes_per_launch"] < 1.1 * r["config"]["rows_per_gpu"] * r["config"]["dim"] * 4
        assert roof["traffic"] is None and roof["traffic_rows"] is None
    assert r1["roofline"]["bytes_per_launch"] > r2["roofline"]["bytes_per_launch"]


@pytest.mark.gpu
@pytest.mark.parametrize("collective", ["engine", "torch"])
def test_rccl_one_rank_gather_equals_plain(tmp_path, collective):
    """The driver's N>1 runs initialise RCCL and all-gather every step; a
    one-GPU box cannot host two RCCL ranks, so this forces the process group,
    the barrier / MAX all-reduce of the timing and the all-gather + on-device
    merge at world size 1 (VS_BENCH_FORCE_DIST) under torch.distributed.run
    with the nccl backend, and checks the keys against the plain run. Both
    exchanges: the engine's communicator (vs_gather_merge_keys, the default)
    and torch.distributed's all-gather + vs_merge_keys."""
    extra = ["--config", "c3", "--rows", "200000"]
    r1, k1 = _bench(tmp_path, "plain", 1, extra)
    out = str(tmp_path / f"rccl_{collective}.npy")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), "bench.py",
           "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-secondary",
           "--dump-keys", out] + extra
    env = dict(os.environ, VS_DIST_BACKEND="nccl", VS_BENCH_FORCE_DIST="1",
               VS_COLLECTIVE=collective, MASTER_ADDR="127.0.0.1")
    p = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-3000:]
    r2 = json.loads([l for l in p.stdout.splitlines() if l.startswith("{")][-1])
    assert r2["n_gpus"] == 1 and r2["config"]["rows_per_gpu"] == 200_000
    assert r2["config"]["collective"] == collective
    assert r2["roofline"]["traffic"] is None  # no PMC entry at 200k rows
    assert r2["roofline"]["bytes_per_launch"] == r1["roofline"]["bytes_per_launch"]
    np.testing.assert_array_equal(k1, np.load(out))
