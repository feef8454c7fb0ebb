"""bench.py's roofline.traffic is the PMC HBM bytes of ONE launch over the
rank's own share: a committed FETCH_SIZE entry is
reported only for a run whose rows_per_gpu equals the rows that entry was
measured on, so an N > 1 line never carries the N = 1 launch's bytes against
its own (smaller) bytes_per_launch. CPU only: world size 2 over gloo, each
rank building its line's roofline exactly as bench.main does."""
import json
import os
import socket
import sys

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    sys.path.insert(0, ROOT)
    import bench
    return bench


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _entry(bench, key):
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    return d[key]


def test_traffic_only_for_the_measured_rows():
    bench = _bench()
    e = _entry(bench, "c3_i8")
    assert e["rows"] == 10_000_000
    assert bench.pmc_traffic("c3_i8", 10_000_000) == e["hbm_bytes_per_launch"]
    for rows in (5_000_000, 2_500_000, 9_999_999):
        assert bench.pmc_traffic("c3_i8", rows) is None
    # a share measured at its own size has its own entry (key c3_i8@1250000)
    d = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    s = d.get("c3_i8@1250000")
    want = s["hbm_bytes_per_launch"] if s and s.get("rows") == 1_250_000 else None
    assert bench.pmc_traffic("c3_i8", 1_250_000) == want
    assert bench.pmc_traffic("no_such_config", 10_000_000) is None


def test_one_rank_line_carries_matching_traffic():
    bench = _bench()
    r = bench.scan_roofline("c3", 10_000_000, 768, "bf16", 256, 10, 1.8, True)
    assert r["traffic"] == _entry(bench, "c3_i8")["hbm_bytes_per_launch"]
    assert r["traffic_rows"] == 10_000_000
    # the figure and the algorithmic bytes describe the same launch (no 8x)
    assert 0.99 < r["traffic"] / r["bytes_per_launch"] < 1.05
    assert "bf16_equivalent_throughput_frac" in r and "exact_tflops_vs_bf16_peak" not in r


def _rank(rank, world, port, out):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        bench = _bench()
        import __graft_entry__ as ge
        pkg = ge.load_package()
        from importlib import import_module
        shard = import_module(pkg.__name__ + ".shard")
        n_full = bench.CONFIGS["c3"][0]
        lo, hi = shard.shard_range(n_full, world, rank)
        roof = bench.scan_roofline("c3", hi - lo, 768, "bf16", 256, 10, 0.9, True)
        lines = [None] * world
        dist.all_gather_object(lines, {"rows_per_gpu": hi - lo, "roofline": roof})
        if rank == 0:
            out.put(lines)
    finally:
        dist.destroy_process_group()


def test_two_rank_gloo_line_has_no_foreign_traffic():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    lines = q.get(timeout=180)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for ln in lines:
        assert ln["rows_per_gpu"] == 5_000_000
        r = ln["roofline"]
        assert r["bytes_per_launch"] == 5_000_000 * 768 + 256 * 768 + 256 * 10 * 12
        # no 5M-row entry is committed: null, never the 10M-row launch's 7.7 GB
        assert r["traffic"] is None and r["traffic_rows"] is None
