"""Multi-process (world_size 2, gloo, CPU) test of the row-shard / all-gather /
merge orchestration used by bench.py. The local search and the merge are the
oracle here (the product binds the HIP engine); what is under test is the
sharding arithmetic and the exchange: the union of per-rank top-k lists,
merged, must equal the unsharded top-k."""
import os
import socket

import numpy as np
import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _keys(scores, rows):
    s = np.where(scores == 0, np.float32(0), scores).astype(np.float32).view(np.uint32).astype(np.uint64)
    o = np.where(s & 0x80000000, (~s) & 0xFFFFFFFF, s | 0x80000000).astype(np.uint64)
    return (o << np.uint64(32)) | (np.uint64(0xFFFFFFFF) - rows.astype(np.uint64))


def _worker(rank, world, port, n, dim, nq, k, q, form="torch"):
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import __graft_entry__ as ge
    from importlib import import_module
    from oracle import oracle
    pkg = ge.load_package()
    shard = import_module(pkg.__name__ + ".shard")
    lo, hi = shard.shard_range(n, world, rank)
    X = oracle.generate(oracle.SEED_CORPUS, lo, hi - lo, dim, bf16=True)
    Q = oracle.preprocess(oracle.generate(oracle.SEED_QUERY, 0, nq, dim), True, True)

    def local_search(queries, kk):
        s32, s64, rows, cnt = oracle.search(X, queries.numpy(), kk, row_base=lo)
        return torch.from_numpy(_keys(s32, rows).view(np.int64))

    def merge(gathered, kk):
        g = gathered.numpy().view(np.uint64).reshape(gathered.shape[0], -1, gathered.shape[2])
        out = np.sort(np.concatenate(list(g), axis=1), axis=1)[:, ::-1][:, :kk]
        return torch.from_numpy(np.ascontiguousarray(out).view(np.int64))

    if form == "torch":
        ss = shard.ShardedSearch(local_search, merge)
    else:
        # the engine form's dispatch (engine_gather_merge binds
        # vs_gather_merge_keys): one callable exchanges and merges, and the
        # torch all-gather + `merge` pair must not run
        def gather_merge(local, kk):
            flat = torch.empty((world * local.shape[0], local.shape[1]), dtype=local.dtype)
            dist.all_gather_into_tensor(flat, local.contiguous())
            return merge(flat.view(world, local.shape[0], local.shape[1]), kk)

        def no_merge(gathered, kk):
            raise AssertionError("torch exchange used with gather_merge set")

        ss = shard.ShardedSearch(local_search, no_merge, gather_merge=gather_merge,
                                 world_size=world)
    res = ss.search(torch.from_numpy(Q), k).numpy().view(np.uint64)
    q.put((rank, res))
    dist.destroy_process_group()


def test_shard_ranges_cover_exactly():
    import __graft_entry__ as ge
    from importlib import import_module
    shard = import_module(ge.load_package().__name__ + ".shard")
    for n in (0, 1, 7, 10_000_000, 100_000_001):
        for P in (1, 2, 3, 4, 8):
            rs = [shard.shard_range(n, P, p) for p in range(P)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            assert max(h - l for l, h in rs) - min(h - l for l, h in rs) <= -(-n // P)


@pytest.mark.timeout(300)
@pytest.mark.parametrize("form", ["torch", "gather_merge"])
def test_two_rank_gloo_merge_equals_unsharded(orc, form):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    n, dim, nq, k, world = 6001, 128, 5, 10, 2
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, dim, nq, k, q, form)) for r in range(world)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
    Q = orc.preprocess(orc.generate(orc.SEED_QUERY, 0, nq, dim), True, True)
    s32, s64, rows, cnt = orc.search(X, Q, k)
    ref = _keys(s32, rows)
    assert np.array_equal(got[0], ref) and np.array_equal(got[1], ref)


def test_exchange_stream_needs_a_result_ring():
    """with an exchange stream, batch i's pooled local keys would be
    overwritten by batch i + 1's search while batch i's exchange still reads
    them unless the results rotate over a ring (>= 2) the search stream waits
    through; a ring-less configuration is refused before anything runs."""
    import __graft_entry__ as ge
    from importlib import import_module
    pkg = ge.load_package()
    shard = import_module(pkg.__name__ + ".shard")
    calls = []
    sh = shard.ShardedSearch(local_search=lambda q, k: calls.append("local"),
                             merge=lambda g, k: None,
                             gather_merge=lambda l, k: calls.append("gather"),
                             world_size=2, exchange_stream=object(), exchange_ring=1)
    with pytest.raises(ValueError, match="exchange_ring"):
        sh.search(np.zeros((4, 8), np.float32), 3)
    assert calls == []
