"""vector-service handler mirror end to end on the device: /upsert then /search
through the same JSON the reference exchanges (ingest-service storeVectors,
rag/ingest-service/main.go:359-393; retrieval-service searchVectorDB,
rag/retrieval-service/main.go:219-276), checked against the oracle.

Config 1 of BASELINE.json (regulatory_docs, ~220 chunk embeddings, top_k 5)
is exercised with synthetic 768-d vectors in place of the Gemini embeddings
(not reproducible offline)."""
import json
import threading
import uuid

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def svcmod(pkg):
    from importlib import import_module
    return import_module(pkg.__name__ + ".service")


@pytest.fixture()
def service(pkg, svcmod):
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng)  # reference defaults: 3 x 768 Cosine collections
    yield s
    s.close()
    eng.close()


def _post(s, path, obj):
    st, body, ct = s.handle("POST", path, json.dumps(obj).encode())
    return st, body, ct


def _ids(n, seed=0):
    rng = np.random.default_rng(seed)
    return [str(uuid.UUID(bytes=rng.bytes(16), version=4)) for _ in range(n)]


def test_routes_and_methods(service):
    st, body, ct = service.handle("GET", "/health")
    h = json.loads(body)
    assert st == 200 and h["status"] == "healthy" and h["service"] == "vector-service"
    assert list(h) == sorted(h) and body.endswith(b"\n")
    st, body, ct = service.handle("GET", "/collections")
    assert st == 200 and body == b'{"collections":["regulatory_docs","merchant_docs","kyc_docs"]}\n'
    for path in ("/collections",):
        st, body, ct = service.handle("POST", path)
        assert (st, body, ct) == (405, b"Method not allowed\n", "text/plain; charset=utf-8")
    for path in ("/upsert", "/search"):
        st, body, ct = service.handle("GET", path)
        assert (st, body) == (405, b"Method not allowed\n")
    st, body, ct = service.handle("GET", "/nope")
    assert (st, body) == (404, b"404 page not found\n")


def test_config1_regulatory_docs(service, orc):
    """~220 chunk vectors upserted as ingest-service does, searched top_k 5."""
    n, dim = 220, 768
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim) * 3.0  # not unit: exercises the cosine preprocess
    ids = _ids(n)
    for lo in range(0, n, 100):  # ingest batches
        pts = [{"id": ids[i], "vector": X[i].tolist(),
                "payload": {"text": f"chunk <{i}> & more", "document_id": "doc-1", "position": i}}
               for i in range(lo, min(n, lo + 100))]
        st, body, _ = _post(service, "/upsert", {"collection": "regulatory_docs", "points": pts})
        assert st == 200, body
        assert json.loads(body) == {"collection": "regulatory_docs", "points": len(pts),
                                    "status": "success"}
    Q = orc.generate(orc.SEED_QUERY, 0, 8, dim)
    Xp = orc.preprocess(X, True)
    for qi in range(8):
        # the query goes over the wire as JSON numbers decoded straight to float32
        st, body, _ = _post(service, "/search", {"collection": "regulatory_docs",
                                                 "query": Q[qi].tolist(), "top_k": 5,
                                                 "filter": {}})
        assert st == 200, body
        assert body.endswith(b"\n")
        res = json.loads(body)
        assert res["count"] == 5 and len(res["results"]) == 5
        assert list(res["results"][0]) == ["id", "score", "payload"]
        rows = np.array([[ids.index(r["id"]) for r in res["results"]]], np.uint64)
        scores = np.array([[r["score"] for r in res["results"]]])
        qp = orc.preprocess(Q[qi:qi + 1], True)
        s32, s64, rr, cc = orc.search(Xp, qp, 5)
        resc = orc.rescore(Xp, qp, rows, np.array([5], np.uint32))
        assert not orc.check_topk(scores, rows, np.array([5]), s64, rr, cc, resc, 1e-5)
        # score is float64(float32): exactly representable as f32
        assert all(np.float64(np.float32(x)) == x for x in scores[0])
        top = res["results"][0]
        i = ids.index(top["id"])
        assert top["payload"] == {"document_id": "doc-1", "position": i,
                                  "text": f"chunk <{i}> & more"}
    # raw bytes: payload keys sorted, HTML escaped
    assert b'"payload":{"document_id":"doc-1","position":' in body
    assert b"\\u003c" in body and b"\\u0026" in body


def test_default_topk_and_overwrite(service, orc):
    dim = 768
    X = orc.generate(7, 0, 12, dim)
    ids = _ids(12, seed=3)
    _post(service, "/upsert", {"collection": "kyc_docs",
                               "points": [{"id": ids[i], "vector": X[i].tolist()} for i in range(12)]})
    st, body, _ = _post(service, "/search", {"collection": "kyc_docs", "query": X[4].tolist()})
    res = json.loads(body)
    assert res["count"] == 5 and res["results"][0]["id"] == ids[4]   # TopK 0 -> 5
    assert res["results"][0]["payload"] == {}
    # overwrite point 4 by id (upper-case UUID input, canonical lower-case output)
    st, body, _ = _post(service, "/upsert", {"collection": "kyc_docs", "points": [
        {"id": ids[4].upper(), "vector": (-X[4]).tolist(), "payload": {"v": 2}}]})
    assert st == 200
    st, body, _ = _post(service, "/search", {"collection": "kyc_docs", "query": X[4].tolist(),
                                             "top_k": 12})
    res = json.loads(body)
    assert res["count"] == 12
    assert res["results"][-1]["id"] == ids[4] and res["results"][-1]["payload"] == {"v": 2}
    assert abs(res["results"][-1]["score"] + 1.0) < 1e-5


def test_errors(service):
    up = lambda pts, coll="merchant_docs": _post(service, "/upsert", {"collection": coll, "points": pts})
    assert up([{"id": 5, "vector": [0.0] * 768}]) == (400, b'{"error":"Point ID must be a string"}\n',
                                                       "application/json")
    assert up([{"id": "x"}])[:2] == (400, b'{"error":"Point vector must be provided"}\n')
    assert up([{"id": "x", "vector": "no"}])[:2] == (400, b'{"error":"point vector must be an array"}\n')
    assert up([{"id": "x", "vector": [1, "a"]}])[:2] == (400, b'{"error":"vector contains non-numeric value"}\n')
    assert _post(service, "/upsert", {"points": []})[:2] == (400, b'{"error":"Collection name required"}\n')
    st, body, _ = service.handle("POST", "/upsert", b"{bad")
    assert (st, body) == (400, b'{"error":"Invalid request body"}\n')
    st, body, _ = up([{"id": "not-a-uuid", "vector": [0.0] * 768}])
    assert st == 500 and body.startswith(b'{"error":"Failed to upsert: ')
    st, body, _ = up([{"id": _ids(1)[0], "vector": [0.1, 0.2, 0.3]}])
    assert st == 500 and b"expected dim: 768, got 3" in body
    st, body, _ = up([{"id": _ids(1)[0], "vector": [0.0] * 768}], coll="nope")
    assert st == 500 and b"Not found: Collection `nope` doesn't exist!" in body
    # README.md:725-738's 3-d probe against a 768-d collection: an engine error, not results
    st, body, _ = _post(service, "/search", {"collection": "regulatory_docs", "query": [0.1, 0.2, 0.3],
                                             "top_k": 1})
    assert st == 500 and body.startswith(b'{"error":"Search failed: ')
    st, body, _ = _post(service, "/search", {"collection": "nope", "query": [0.0] * 768})
    assert st == 500 and b"Not found" in body
    st, body, _ = service.handle("POST", "/search", b'{"query":"x"}')
    assert (st, body) == (400, b'{"error":"Invalid request body"}\n')
    # empty collection: results is [] (make([]SearchResult, 0)), not null
    st, body, _ = _post(service, "/search", {"collection": "merchant_docs", "query": [0.5] * 768})
    assert (st, body) == (200, b'{"results":[],"count":0}\n')


def test_concurrent_search_and_upsert(service, orc):
    dim = 768
    X = orc.generate(11, 0, 400, dim)
    ids = _ids(400, seed=9)
    _post(service, "/upsert", {"collection": "merchant_docs",
                               "points": [{"id": ids[i], "vector": X[i].tolist()} for i in range(200)]})
    errors = []

    def searcher(t):
        for j in range(10):
            q = X[(t * 10 + j) % 200]
            st, body, _ = _post(service, "/search", {"collection": "merchant_docs",
                                                     "query": q.tolist(), "top_k": 3})
            r = json.loads(body)
            if st != 200 or r["results"][0]["id"] != ids[(t * 10 + j) % 200]:
                errors.append((t, j, st, body[:200]))

    def upserter():
        for lo in range(200, 400, 50):
            st, body, _ = _post(service, "/upsert", {"collection": "merchant_docs", "points": [
                {"id": ids[i], "vector": X[i].tolist()} for i in range(lo, lo + 50)]})
            if st != 200:
                errors.append(("up", st, body))

    th = [threading.Thread(target=searcher, args=(t,)) for t in range(6)] + [threading.Thread(target=upserter)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors[:3]
    st, body, _ = _post(service, "/search", {"collection": "merchant_docs", "query": X[399].tolist(),
                                             "top_k": 1})
    assert json.loads(body)["results"][0]["id"] == ids[399]


# ------------------------------------------------------------ dynamic batcher
_BATCH_CFG = {"collections": [{"name": "b16", "dim": 768, "metric": "Cosine", "dtype": "bf16"},
                              {"name": "f32", "dim": 768, "metric": "Cosine", "dtype": "f32"}]}


def _fill(s, orc, coll, n, seed, bf16):
    X = orc.generate(seed, 0, n, 768)
    ids = _ids(n, seed=seed)
    for lo in range(0, n, 512):
        st, body, _ = _post(s, "/upsert", {"collection": coll, "points": [
            {"id": ids[i], "vector": X[i].tolist(), "payload": {"i": i}}
            for i in range(lo, min(n, lo + 512))]})
        assert st == 200, body
    return orc.preprocess(X, True, bf16), ids


@pytest.fixture(params=[0])
def batch_service(pkg, svcmod, request):
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, dict(_BATCH_CFG, batching={"max_wait_us": request.param}))
    yield s
    s.close()
    eng.close()


@pytest.mark.parametrize("batch_service", [50_000], indirect=True)
def test_batcher_concurrent_requests_exact(batch_service, orc):
    """64 concurrent /search requests over two collections with mixed k
    (including k > 128, the GEMV class) are coalesced into few engine calls,
    and every reply is still that request's own exact top k. (Python clients
    serialise on the GIL while they build their bodies, so the batcher
    lingers 50 ms here to collect them.)"""
    s = batch_service
    data = {"b16": _fill(s, orc, "b16", 3000, 21, True), "f32": _fill(s, orc, "f32", 2000, 22, False)}
    nreq = 64
    Q = orc.generate(orc.SEED_QUERY, 500, nreq, 768)
    ks = [1 + (7 * i) % 60 for i in range(nreq)]
    ks[5], ks[40] = 200, 129
    colls = ["b16" if i % 3 else "f32" for i in range(nreq)]
    replies = [None] * nreq
    gate = threading.Barrier(nreq)

    def client(i):
        gate.wait()
        replies[i] = _post(s, "/search", {"collection": colls[i], "query": Q[i].tolist(),
                                          "top_k": ks[i], "filter": None})

    th = [threading.Thread(target=client, args=(i,)) for i in range(nreq)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for i in range(nreq):
        st, body, _ = replies[i]
        assert st == 200, body
        res = json.loads(body)
        Xp, ids = data[colls[i]]
        k = ks[i]
        assert res["count"] == k == len(res["results"])
        rows = np.array([[ids.index(r["id"]) for r in res["results"]]], np.uint64)
        assert all(r["payload"] == {"i": int(rows[0, j])} for j, r in enumerate(res["results"]))
        scores = np.array([[r["score"] for r in res["results"]]])
        qp = orc.preprocess(Q[i:i + 1], True, colls[i] == "b16")
        s32, s64, rr, cc = orc.search(Xp, qp, k)
        resc = orc.rescore(Xp, qp, rows, np.array([k], np.uint32))
        assert not orc.check_topk(scores, rows, np.array([k]), s64, rr, cc, resc, 1e-5), i
    st = s.stats()
    assert st["batching"]["enabled"] and st["requests"] >= nreq
    assert st["engine_calls"] < st["requests"] and st["largest_call"] >= 2, st


def test_batcher_disabled(pkg, svcmod, orc):
    eng = pkg.VectorEngine(device=0)
    cfg = dict(_BATCH_CFG, batching={"enabled": False})
    s = svcmod.VectorService(eng, cfg)
    try:
        Xp, ids = _fill(s, orc, "b16", 300, 5, True)
        st, body, _ = _post(s, "/search", {"collection": "b16", "query": Xp[7].tolist(), "top_k": 3})
        assert st == 200 and json.loads(body)["results"][0]["id"] == ids[7]
        assert s.stats() == {"batching": {"enabled": False, "max_batch": 256, "max_wait_us": 0,
                                          "workers": 2, "lead_us": 300,
                                          "caller_runs": True},
                             "requests": 0, "engine_calls": 0, "largest_call": 0,
                             "calls_by_log2_nq": [0] * 10}
    finally:
        s.close()
        eng.close()
    with pytest.raises(Exception):
        svcmod.VectorService(pkg.VectorEngine(device=0), dict(_BATCH_CFG, batching={"max_batch": 0}))


def test_loadgen_closed_loop(batch_service, orc):
    """C5-shaped load in miniature: 32 closed-loop clients, k in [3, 50],
    two collections; no errors, and the batcher forms multi-query calls."""
    s = batch_service
    _fill(s, orc, "b16", 2000, 31, True)
    _fill(s, orc, "f32", 1000, 32, False)
    rep = s.loadgen(["b16", "f32"], 768, clients=32, seconds=1.5, k_min=3, k_max=50)
    assert rep["errors"] == 0, rep["first_error"]
    assert rep["requests"] > 100 and rep["qps"] > 0
    assert rep["lat_ms"]["p50"] <= rep["lat_ms"]["p99"] <= rep["lat_ms"]["max"]
    st = s.stats()
    assert st["requests"] == rep["requests"] and st["largest_call"] >= 2, st


def test_bulk_generate_ids_and_overwrite(batch_service, orc):
    """vsvc_bulk_generate: device-generated points with synthetic v4 UUIDs,
    searchable, overwritable by id; new ids append after them."""
    import re
    s = batch_service
    n = 5000
    s.bulk_generate("b16", n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, 768, bf16=True)
    uid = s.point_id("b16", 123)
    assert re.fullmatch(r"[0-9a-f]{8}-[0-9a-f]{4}-4[0-9a-f]{3}-[89ab][0-9a-f]{3}-[0-9a-f]{12}", uid)
    assert len({s.point_id("b16", r) for r in (0, 1, 123, n - 1)}) == 4
    st, body, _ = _post(s, "/search", {"collection": "b16", "query": X[123].tolist(), "top_k": 3})
    res = json.loads(body)
    assert st == 200 and res["results"][0]["id"] == uid and res["results"][0]["payload"] == {}
    # overwrite the bulk point by its id (upper case in, canonical out)
    st, body, _ = _post(s, "/upsert", {"collection": "b16", "points": [
        {"id": uid.upper(), "vector": (-X[123]).tolist(), "payload": {"v": 1}}]})
    assert st == 200, body
    st, body, _ = _post(s, "/search", {"collection": "b16", "query": (-X[123]).tolist(), "top_k": 1})
    r0 = json.loads(body)["results"][0]
    assert r0["id"] == uid and r0["payload"] == {"v": 1}
    # a new id appends at row n
    new = _ids(1, seed=77)[0]
    st, body, _ = _post(s, "/upsert", {"collection": "b16", "points": [
        {"id": new, "vector": X[7].tolist(), "payload": {"new": True}}]})
    assert st == 200 and s.point_id("b16", n) == new
    st, body, _ = _post(s, "/search", {"collection": "b16", "query": X[7].tolist(), "top_k": 2})
    got = {r["id"] for r in json.loads(body)["results"]}
    assert got == {new, s.point_id("b16", 7)}
    with pytest.raises(Exception):
        s.bulk_generate("b16", 10, 1)  # only into an empty collection


def test_filter_modes(pkg, svcmod, orc):
    """Default "ignore": `filter` is decoded and dropped, as the reference does.
    "match": only points whose payload equals every filter entry are eligible
    (the pre-mask runs inside the scan); cached masks follow upserts."""
    n, dim = 3000, 768
    X = orc.generate(41, 0, n, dim)
    ids = _ids(n, seed=41)
    docs = ["doc-a", "doc-b", "doc-c"]
    pts = [{"id": ids[i], "vector": X[i].tolist(),
            "payload": {"document_id": docs[i % 3], "lang": "en" if i % 2 else "de", "n": i % 5}}
           for i in range(n)]
    Xp = orc.preprocess(X, True, True)
    Q = orc.generate(orc.SEED_QUERY, 41, 6, dim)
    for mode in ("ignore", "match"):
        eng = pkg.VectorEngine(device=0)
        s = svcmod.VectorService(eng, {"collections": [{"name": "c", "dim": dim, "dtype": "bf16"}],
                                       "filter": mode})
        try:
            for lo in range(0, n, 1000):
                assert _post(s, "/upsert", {"collection": "c", "points": pts[lo:lo + 1000]})[0] == 200
            for flt, pred in (({"document_id": "doc-b"}, lambda i: i % 3 == 1),
                              ({"document_id": "doc-a", "lang": "en"}, lambda i: i % 6 == 3),
                              ({"n": 2}, lambda i: i % 5 == 2),          # number: float64 equality
                              ({"n": "2"}, lambda i: False),             # string != number
                              ({}, lambda i: True)):
                mask = np.array([pred(i) or mode == "ignore" for i in range(n)])
                for qi in range(len(Q)):
                    st, body, _ = _post(s, "/search", {"collection": "c", "query": Q[qi].tolist(),
                                                       "top_k": 8, "filter": flt})
                    assert st == 200, body
                    res = json.loads(body)["results"]
                    rows = [ids.index(r["id"]) for r in res]
                    idx = np.flatnonzero(mask)
                    qp = orc.preprocess(Q[qi:qi + 1], True, True)
                    s32, s64, rr, cc = orc.search(np.ascontiguousarray(Xp[idx]), qp, 8)
                    exp = idx[rr[0, :cc[0]].astype(np.int64)].tolist()
                    assert rows == exp, (mode, flt, qi)
            if mode == "match":  # payload change -> the cached doc-b mask must not be reused
                assert _post(s, "/upsert", {"collection": "c", "points": [
                    {"id": ids[0], "vector": X[0].tolist(), "payload": {"document_id": "doc-b"}}]})[0] == 200
                st, body, _ = _post(s, "/search", {"collection": "c", "query": X[0].tolist(),
                                                   "top_k": 1, "filter": {"document_id": "doc-b"}})
                assert json.loads(body)["results"][0]["id"] == ids[0]
        finally:
            s.close()
            eng.close()
    with pytest.raises(Exception):
        svcmod.VectorService(pkg.VectorEngine(device=0), {"collections": [], "filter": "maybe"})


def test_filter_cache_eviction_and_resident_filters(pkg, svcmod, orc):
    """"match" mode keeps one device-resident filter per cached filter; more
    distinct filters than the cache holds (64) evict and drop them, repeated
    filters reuse them, and an upsert that adds rows makes them stale. Every
    reply must hold only points whose payload matches, best first, and equal
    the oracle's top k over the matching points."""
    n, dim, groups = 2600, 128, 70
    X = orc.generate(43, 0, n, dim)
    ids = _ids(n, seed=43)
    pts = [{"id": ids[i], "vector": X[i].tolist(), "payload": {"g": i % groups}}
           for i in range(n)]
    Xp = orc.preprocess(X, True, False)
    Q = orc.generate(orc.SEED_QUERY, 43, 3, dim)
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, {"collections": [{"name": "c", "dim": dim}], "filter": "match"})
    try:
        assert _post(s, "/upsert", {"collection": "c", "points": pts})[0] == 200

        grp = [i % groups for i in range(n)]

        def check(g, qi, nrows):
            st, body, _ = _post(s, "/search", {"collection": "c", "query": Q[qi].tolist(),
                                               "top_k": 5, "filter": {"g": g}})
            assert st == 200, body
            got = [ids.index(r["id"]) for r in json.loads(body)["results"]]
            idx = np.array([i for i in range(nrows) if grp[i] == g])
            s32, s64, rr, cc = orc.search(np.ascontiguousarray(Xp[idx]), orc.preprocess(
                Q[qi:qi + 1], True, False), 5)
            assert got == idx[rr[0, :cc[0]].astype(np.int64)].tolist(), (g, qi)

        for rnd in range(2):  # 70 distinct filters twice: evictions, then reuse
            for g in range(groups):
                check(g, (g + rnd) % 3, n)
        extra = [{"id": str(uuid.UUID(int=(1 << 100) + i, version=4)), "vector": X[i].tolist(),
                  "payload": {"g": i % groups}} for i in range(100)]
        assert _post(s, "/upsert", {"collection": "c", "points": extra})[0] == 200
        ids.extend(p["id"] for p in extra)
        grp.extend(i % groups for i in range(100))
        X2 = np.concatenate([X, X[:100]])
        Xp = orc.preprocess(X2, True, False)
        for g in (0, 5, 69):
            check(g, 1, n + 100)
    finally:
        s.close()
        eng.close()


def test_batcher_groups_filtered_requests(pkg, svcmod, orc):
    """"match" mode with batching: concurrent requests that share a filter go
    to the engine together (one vs_search_filter_id call per filter group:
    the MFMA pass with the bitmap fused for a dense filter, gathers for a
    selective one), and each reply is still its own exact top k over the
    matching points."""
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, dict(_BATCH_CFG, filter="match",
                                       batching={"max_wait_us": 50_000}))
    try:
        n = 4000
        X = orc.generate(47, 0, n, 768)
        ids = _ids(n, seed=47)
        for lo in range(0, n, 500):
            st, body, _ = _post(s, "/upsert", {"collection": "b16", "points": [
                {"id": ids[i], "vector": X[i].tolist(), "payload": {"g": i % 2, "h": i % 40}}
                for i in range(lo, min(n, lo + 500))]})
            assert st == 200, body
        Xp = orc.preprocess(X, True, True)
        flts = [{"g": 1}, {"h": 7}, {"g": 0, "h": 4}]
        preds = [lambda i: i % 2 == 1, lambda i: i % 40 == 7, lambda i: i % 2 == 0 and i % 40 == 4]
        nreq = 48
        Q = orc.generate(orc.SEED_QUERY, 700, nreq, 768)
        ks = [1 + (5 * i) % 30 for i in range(nreq)]
        replies = [None] * nreq
        for f in flts:  # build (and make resident) every filter before the burst
            assert _post(s, "/search", {"collection": "b16", "query": Q[0].tolist(),
                                        "top_k": 1, "filter": f})[0] == 200
        before = s.stats()
        gate = threading.Barrier(nreq)

        def client(i):
            gate.wait()
            replies[i] = _post(s, "/search", {"collection": "b16", "query": Q[i].tolist(),
                                              "top_k": ks[i], "filter": flts[i % 3]})

        th = [threading.Thread(target=client, args=(i,)) for i in range(nreq)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for i in range(nreq):
            st, body, _ = replies[i]
            assert st == 200, body
            res = json.loads(body)["results"]
            rows = [ids.index(r["id"]) for r in res]
            idx = np.array([j for j in range(n) if preds[i % 3](j)])
            s32, s64, rr, cc = orc.search(np.ascontiguousarray(Xp[idx]), orc.preprocess(
                Q[i:i + 1], True, True), ks[i])
            exp = idx[rr[0, :cc[0]].astype(np.int64)].tolist()
            assert rows == exp, i
        after = s.stats()
        calls = after["engine_calls"] - before["engine_calls"]
        reqs = after["requests"] - before["requests"]
        assert reqs == nreq and calls < reqs, (before, after)
    finally:
        s.close()
        eng.close()


def test_negative_top_k_is_a_bad_request(service):
    """uint64(req.TopK) would wrap a negative top_k to a limit near 2^64 (its
    Qdrant reply is unpinned); the mirror answers 400."""
    q = [0.1] * 768
    st, body, _ = _post(service, "/search", {"collection": "kyc_docs", "query": q, "top_k": -3})
    assert (st, body) == (400, b'{"error":"top_k must not be negative"}\n')
    st, body, _ = _post(service, "/search", {"collection": "kyc_docs", "query": q, "top_k": 0})
    assert st == 200 and json.loads(body) == {"results": [], "count": 0}
