"""Whole collections placed per device (VS_FLAG_PLACE_COLLECTIONS).

A vs_open_multi engine with the flag keeps every collection whole on one of
its devices (the least loaded at creation) and sends each call to that
device's engine alone: calls for collections on different devices run
concurrently and no collective runs (the reference serves its three
collections from concurrent handlers, rag/vector-service/main.go:77,
:80-119). On the one-GPU box the engine's two shards share device 0, so
every collection lands there; every entry point must answer exactly as a
single-device engine does (the cross-device copies of vs_search_keys run only
on a multi-GPU node).
"""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def placed(pkg):
    eng = pkg.VectorEngine(shards=[0, 0], place_collections=True)
    yield eng
    eng.close()


def test_placement_layout(placed, pkg):
    assert placed.layout() == (2, 1)
    for i in range(3):
        placed.create_collection(f"p{i}", 128, 0, 1, 1000)
        assert placed.placement(f"p{i}") == 0
    placed.create_collection("pb", 128, 0, 1, 0, 500)  # a placed collection takes a row_base
    with pytest.raises(pkg.VSError):
        placed.create_collection("p0", 128, 0, 1)  # exists
    for nm in ("p0", "p1", "p2", "pb"):
        placed.drop_collection(nm)
    with pytest.raises(pkg.VSError):
        placed.placement("p0")
    striped = pkg.VectorEngine(shards=[0, 0])
    try:
        striped.create_collection("s", 64, 0, 1)
        assert striped.placement("s") == 0  # one distinct device
    finally:
        striped.close()


@pytest.mark.parametrize("dtype", [0, 1])
def test_placed_equals_single_device(placed, engine, orc, pkg, dtype, tmp_path):
    dim, n = 768, 60_000
    name = f"pl{dtype}"
    for e in (placed, engine):
        e.create_collection(name, dim, 0, dtype, n)
        e.generate(name, n, orc.SEED_CORPUS)
    try:
        assert placed.collection_info(name) == engine.collection_info(name)
        Q = orc.generate(orc.SEED_QUERY, 9, 64, dim)
        for nq, k in ((1, 10), (64, 10), (5, 100), (2, 1500)):
            a = placed.search(name, Q[:nq], k)
            b = engine.search(name, Q[:nq], k)
            assert all(np.array_equal(x, y) for x, y in zip(a, b)), (nq, k)
        allow = np.random.default_rng(1).random(n) < 0.03
        a = placed.search_filtered(name, Q[:3], 20, allow)
        b = engine.search_filtered(name, Q[:3], 20, allow)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
        fid = placed.filter_create(name, allow)
        c = placed.search_filter_id(name, Q[:3], 20, fid)
        assert all(np.array_equal(x, y) for x, y in zip(c, b))
        placed.filter_drop(fid)
        with pytest.raises(pkg.VSError):
            placed.search_filter_id(name, Q[:3], 20, fid)
        assert placed.checksum(name) == engine.checksum(name)
        assert np.array_equal(placed.read_rows(name, 123, 7), engine.read_rows(name, 123, 7))
        # device-pointer search on the engine's first device
        import torch
        dq = torch.from_numpy(Q[:8]).cuda()
        dk = torch.zeros((8, 10), dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        placed.search_keys(name, dq.data_ptr(), 8, dim, 10, dk.data_ptr(), st)
        torch.cuda.synchronize()
        s, r, c = pkg.keys_decode(dk.cpu().numpy().view(np.uint64))
        want = engine.search(name, Q[:8], 10)
        assert np.array_equal(r, want[1]) and np.array_equal(s, want[0])
        # snapshot of a placed collection restores anywhere, and back
        path = str(tmp_path / f"{name}.snap")
        placed.snapshot(name, path)
        engine.restore(name + "_r", path)
        assert engine.checksum(name + "_r") == engine.checksum(name)
        engine.drop_collection(name + "_r")
        placed.restore(name + "_r", path)
        assert placed.placement(name + "_r") == 0
        assert placed.checksum(name + "_r") == engine.checksum(name)
        a = placed.search(name + "_r", Q[:4], 10)
        b = engine.search(name, Q[:4], 10)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
        placed.drop_collection(name + "_r")
        # upsert into a placed collection (overwrite + append)
        V = orc.generate(77, 0, 3, dim)
        for e in (placed, engine):
            e.upsert(name, [5, n, n + 1], V)
        a = placed.search(name, V, 1)
        b = engine.search(name, V, 1)
        assert all(np.array_equal(x, y) for x, y in zip(a, b))
        assert a[1][:, 0].tolist() == [5, n, n + 1]
    finally:
        for e in (placed, engine):
            e.drop_collection(name)


def test_service_over_placed_engine(pkg, orc):
    """The handler mirror over a placed engine: collections created by the
    service are placed, the batcher keys its lanes on their device, and
    concurrent requests of three collections are answered exactly."""
    import threading
    from importlib import import_module
    svcmod = import_module(pkg.__name__ + ".service")
    names = ["regulatory_docs", "merchant_docs", "kyc_docs"]
    eng = pkg.VectorEngine(shards=[0, 0], place_collections=True)
    cfg = {"collections": [{"name": nm, "dim": 256, "metric": "Cosine", "dtype": "bf16"}
                           for nm in names]}
    s = svcmod.VectorService(eng, cfg)
    ref = pkg.VectorEngine(device=0)
    try:
        for i, nm in enumerate(names):
            s.bulk_generate(nm, 30_000, 11 + i)
            ref.create_collection(nm, 256, 0, 1)
            ref.generate(nm, 30_000, 11 + i)
            assert eng.placement(nm) == 0
        assert s.stats()["batching"]["workers"] == 2  # one device: one lane
        Q = orc.generate(orc.SEED_QUERY, 0, 48, 256)
        out = [None] * 48

        def client(i):
            body = json.dumps({"collection": names[i % 3], "query": Q[i].tolist(),
                               "top_k": 7}).encode()
            out[i] = s.handle("POST", "/search", body)

        th = [threading.Thread(target=client, args=(i,)) for i in range(48)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for i in range(48):
            st, body, _ = out[i]
            assert st == 200
            res = json.loads(body)
            rows = [int(h["id"].replace("-", ""), 16) & ((1 << 62) - 1) for h in res["results"]]
            sc, rr, cc = ref.search(names[i % 3], Q[i], 7)
            assert rows == rr[0].tolist()
    finally:
        s.close()
        eng.close()
        ref.close()
