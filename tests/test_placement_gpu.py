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
        # all-ones sentinel: a slot the search never wrote reads as ~0, not as
        # an empty key (0), so a stream-ordering hole and an empty answer differ
        dk = torch.full((8, 10), -1, dtype=torch.int64, device="cuda")
        st = torch.cuda.current_stream().cuda_stream
        placed.search_keys(name, dq.data_ptr(), 8, dim, 10, dk.data_ptr(), st)
        torch.cuda.synchronize()
        got = dk.cpu().numpy().view(np.uint64)
        assert not np.any(got == np.uint64(0xFFFFFFFFFFFFFFFF)), "keys never written"
        s, r, c = pkg.keys_decode(got)
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


def test_one_hip_runtime(pkg):
    """The process holds one HIP runtime, torch's and the library's alike
    (engine.load_library imports torch first): the round-3 failure above was
    a second runtime whose null stream is not torch's."""
    import torch  # noqa: F401
    from importlib import import_module
    eng_mod = import_module(pkg.__name__ + ".engine")
    assert len(eng_mod.hip_runtimes()) == 1, eng_mod.hip_runtimes()
    assert pkg.load_library().vs_runtime_check() == 0


@pytest.mark.parametrize("dtype", [0, 1])
def test_placed_off_first_device(engine, orc, pkg, dtype):
    """VS_FLAG_ENGINE_PER_SHARD: shards [0, 0] are two device engines on the
    one GPU, so a collection lands on engine index 1 and vs_search_keys takes
    placed_search_keys (vs_api.cpp: the queries copied from the caller's
    device to the home device after an event on the caller's stream, the keys
    copied back and the caller's stream made to wait on them) -- the path a
    multi-GPU node runs for C5's collections, otherwise unreachable here.
    Checked against a single-device engine and the streaming oracle, on
    torch's null stream and on a side stream. Anchor: three collections
    served concurrently, rag/vector-service/main.go:77, :80-119."""
    import torch
    dim, n = 768, 60_000
    eng2 = pkg.VectorEngine(shards=[0, 0], place_collections=True, engine_per_shard=True)
    name = f"off{dtype}"
    try:
        assert eng2.layout() == (2, 2)
        eng2.create_collection("first", 128, 0, dtype, 0)  # engine 0
        eng2.create_collection(name, dim, 0, dtype, 0)     # engine 1 (fewest collections)
        h = json.loads(eng2.health())
        assert [d["collections"] for d in h["devices"]] == [1, 1], h
        assert eng2.placement(name) == 0  # the device ordinal: both engines are on GPU 0
        eng2.generate(name, n, orc.SEED_CORPUS)
        engine.create_collection(name, dim, 0, dtype, n)
        engine.generate(name, n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 21, 40, dim)
        Qp = orc.preprocess(Q, cosine=True, bf16=bool(dtype))
        for nq, k in ((1, 10), (8, 10), (40, 50), (3, 200)):
            a = eng2.search(name, Q[:nq], k)
            b = engine.search(name, Q[:nq], k)
            assert all(np.array_equal(x, y) for x, y in zip(a, b)), (nq, k)
        side = torch.cuda.Stream()
        for st in (torch.cuda.default_stream(), side):
            with torch.cuda.stream(st):
                for nq, k in ((8, 10), (40, 100), (1, 5)):
                    dq = torch.from_numpy(Q[:nq]).cuda()
                    dk = torch.full((nq, k), -1, dtype=torch.int64, device="cuda")
                    eng2.search_keys(name, dq.data_ptr(), nq, dim, k, dk.data_ptr(), st.cuda_stream)
                    got = dk.cpu().numpy().view(np.uint64)  # ordered on st (torch's copy)
                    assert not np.any(got == np.uint64(0xFFFFFFFFFFFFFFFF)), "keys never written"
                    s, r, c = pkg.keys_decode(got)
                    want = engine.search(name, Q[:nq], k)
                    assert np.array_equal(r, want[1]) and np.array_equal(s, want[0]), (nq, k)
                    s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp[:nq], k, bool(dtype))
                    resc = orc.rescore_generated(orc.SEED_CORPUS, Qp[:nq], r, c, bool(dtype))
                    bad = orc.check_topk(s, r, c, s64, rr, cc, resc, score_rtol=1e-5)
                    assert not bad, bad[:4]
        torch.cuda.synchronize()
    finally:
        eng2.close()
        try:
            engine.drop_collection(name)
        except pkg.VSError:
            pass


def test_placed_create_drop_race_keeps_balance(pkg):
    """Concurrent create / drop of the same names on a placed engine (ADVICE
    r03): a collection is published only once it exists on its device, and
    only its creating call can withdraw it, so no drop ever takes a
    half-made one, no orphan stays on a device and the per-device
    reservation counters never underflow. After the storm every device holds
    nothing and a fresh create lands by the balance rule."""
    import threading
    eng = pkg.VectorEngine(shards=[0, 0], place_collections=True, engine_per_shard=True)
    errors = []

    def worker(t):
        for i in range(60):
            nm = f"race{(t + i) % 3}"
            try:
                eng.create_collection(nm, 64, 0, 1, 1000)
            except pkg.VSError as e:
                if e.code != -6:  # EXISTS
                    errors.append(("create", e.code, e.msg))
            try:
                eng.drop_collection(nm)
            except pkg.VSError as e:
                if e.code != -2:  # NOT_FOUND
                    errors.append(("drop", e.code, e.msg))

    try:
        th = [threading.Thread(target=worker, args=(t,)) for t in range(6)]
        for x in th:
            x.start()
        for x in th:
            x.join()
        assert not errors, errors[:4]
        for nm in ("race0", "race1", "race2"):
            try:
                eng.drop_collection(nm)
            except pkg.VSError:
                pass
        h = json.loads(eng.health())
        assert [d["collections"] for d in h["devices"]] == [0, 0], h
        eng.create_collection("a", 64, 0, 1, 1000)
        eng.create_collection("b", 64, 0, 1, 1000)
        h = json.loads(eng.health())
        assert [d["collections"] for d in h["devices"]] == [1, 1], h
    finally:
        eng.close()


def test_limit_past_rows_sizes_by_rows(engine, pkg, orc):
    """A limit far past the collection: the host search sizes its
    buffers by min(k, rows) and returns every row, zero past them, in the
    caller's stride k -- no gigabyte allocations for a 300-row collection."""
    dim, n = 128, 300
    engine.create_collection("kclamp", dim, 0, 0)
    try:
        engine.generate("kclamp", n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 0, 2, dim)
        big = 50_000_000  # unclamped: 400 MB of device keys and pinned staging for one query
        k = 400
        s, r, c = engine.search("kclamp", Q, k)
        assert list(c) == [n, n]
        assert np.all(r[:, n:] == 0) and np.all(s[:, n:] == 0)
        want = engine.search("kclamp", Q, n)
        assert np.array_equal(r[:, :n], want[1]) and np.array_equal(s[:, :n], want[0])
        import ctypes
        L = pkg.load_library()
        # one query with a huge k through the C-ABI: the caller's outputs are
        # sized by k (600 MB on the host); the device side must not scale with it
        s1 = np.zeros(big, np.float32)
        r1 = np.zeros(big, np.uint64)
        c1 = np.zeros(1, np.uint32)
        p = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
        q = np.ascontiguousarray(Q[:1], np.float32)
        rc = L.vs_search(engine.handle, b"kclamp", p(q), 1, dim, big, p(s1), p(r1), p(c1))
        assert rc == 0, L.vs_last_error()
        assert int(c1[0]) == n
        assert np.array_equal(r1[:n], want[1][0]) and not np.any(r1[n:n + 1000])
    finally:
        engine.drop_collection("kclamp")
