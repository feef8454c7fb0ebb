"""BASELINE.json configs checked at their own shapes on the device.

* C3 — 10M x 768 bf16, 256-query batches, exact top-10, inner product: the
  batched MFMA path at the production shape (the sample bound, candidate
  capacity and tiles per workgroup all depend on N), against the streaming
  oracle (rows regenerated per thread, no 15 GB host array) on 16 of the 256
  queries, and on all 256 through size-independent properties: full sorted
  lists, every score equal to the exact score of the row it names, and the
  batched answer equal to the single-query GEMV answer (two independent
  kernels) up to the north_star near-tie rule.
* C2 — 1M x 768 fp32 Cosine, single-query GEMV searches, one call each, at
  k = 10 (the rank merge of the waves' lists) and k = 100 (the two-stage
  merge), against the streaming oracle at the fp32 bar (1e-5).
* C5 — multi-collection serving: 3 bf16 collections x 1024-d (bulk
  generated, so the candidate path runs), concurrent /search requests
  through the dynamic batcher with top_k uniform in [3, 50], every reply
  checked against the oracle (UUID -> row through the synthetic bulk ids):
  at 200k rows per collection (one sample tile per workgroup) and at C5's
  own 5M rows (the production 1/64 sample fraction and candidate capacity).

Reference anchor: Points.Search, rag/vector-service/main.go:249-254; the
request body is retrieval-service's searchVectorDB (rag/retrieval-service/
main.go:221-233).
"""
import json
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(orc, s, r, c, s64, rr, cc, resc, tol):
    bad = orc.check_topk(s, r, c, s64, rr, cc, resc, score_rtol=tol)
    assert not bad, bad[:8]


@pytest.mark.timeout(900)
def test_c3_full_size(engine, orc, pkg):
    n, dim, B, k = 10_000_000, 768, 256, 10
    name = "c3_full"
    engine.create_collection(name, dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
    try:
        engine.generate(name, n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 0, B, dim)  # unit queries, as bench.py's
        s, r, c = engine.search(name, Q, k)  # one batch: the MFMA path
        assert np.all(c == k)
        assert np.all(np.diff(s, axis=1) <= 0)
        Qp = orc.preprocess(Q, cosine=False, bf16=True)  # what the engine multiplies
        # every returned score is the exact score of the row it names
        resc = orc.rescore_generated(orc.SEED_CORPUS, Qp, r, c, True)
        assert np.all(np.abs(s - resc) <= 1e-5 * np.abs(resc) + 1e-6)
        # 16 queries against the full streaming oracle
        sel = np.arange(0, B, B // 16)
        s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp[sel], k, True)
        _check(orc, s[sel], r[sel], c[sel], s64, rr, cc, resc[sel], 1e-5)
        # all 256: the batched answer equals the per-query GEMV answer
        # (exact rows, or an exact-score near-tie of them)
        g = [engine.search(name, Q[i:i + 1], k) for i in range(B)]
        gs = np.concatenate([x[0] for x in g])
        gr = np.concatenate([x[1] for x in g])
        gresc = orc.rescore_generated(orc.SEED_CORPUS, Qp, gr, c, True)
        assert np.all(np.abs(gs - gresc) <= 1e-5 * np.abs(gresc) + 1e-6)
        diff = r != gr
        if diff.any():
            band = 1e-5 * np.abs(gresc) + 1e-6
            assert np.all(np.abs(resc[diff] - gresc[diff]) <= band[diff]), \
                "batched and GEMV answers differ beyond near-ties"
        assert diff.mean() < 0.01
        # repeated batches give identical answers
        s2, r2, c2 = engine.search(name, Q, k)
        assert np.array_equal(r2, r) and np.array_equal(s2, s)
    finally:
        engine.drop_collection(name)


def _bulk_row(uuid: str) -> int:
    """Row of a synthetic bulk UUID (vector_service.cpp bulk_uuid)."""
    return int(uuid.replace("-", ""), 16) & ((1 << 62) - 1)


@pytest.mark.timeout(600)
def test_c2_full_size_single_queries(engine, orc, pkg):
    n, dim = 1_000_000, 768
    name = "c2_full"
    engine.create_collection(name, dim, pkg.METRIC_COSINE, pkg.DTYPE_F32, n)
    try:
        engine.generate(name, n, orc.SEED_CORPUS)
        nq = 16
        Q = orc.generate(orc.SEED_QUERY, 7000, nq, dim) * 1.3  # cosine normalises them back
        Qp = orc.preprocess(Q, cosine=True, bf16=False)
        for k in (10, 100):
            got = [engine.search(name, Q[i:i + 1], k) for i in range(nq)]  # one GEMV call each
            s = np.concatenate([g[0] for g in got])
            r = np.concatenate([g[1] for g in got])
            c = np.concatenate([g[2] for g in got])
            assert np.all(c == k)
            s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp, k, False)
            resc = orc.rescore_generated(orc.SEED_CORPUS, Qp, r, c, False)
            _check(orc, s, r, c, s64, rr, cc, resc, 1e-5)
    finally:
        engine.drop_collection(name)


@pytest.mark.timeout(600)
def test_c5_concurrent_mixed_k(pkg, orc):
    _c5_concurrent_mixed_k(pkg, orc, 200_000, 96)


@pytest.mark.timeout(900)
def test_c5_full_size_concurrent_mixed_k(pkg, orc):
    """C5 at its own shape: 3 x 5M x 1024 bf16 (30.7 GB resident), 40
    concurrent requests per collection."""
    _c5_concurrent_mixed_k(pkg, orc, 5_000_000, 120)


def _c5_concurrent_mixed_k(pkg, orc, n, nreq):
    from importlib import import_module
    svcmod = import_module(pkg.__name__ + ".service")
    names = ["regulatory_docs", "merchant_docs", "kyc_docs"]
    dim = 1024
    seeds = {nm: orc.SEED_CORPUS + 17 * i for i, nm in enumerate(names)}
    cfg = {"collections": [{"name": nm, "dim": dim, "metric": "Cosine", "dtype": "bf16"}
                           for nm in names]}
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, cfg)
    try:
        for nm in names:
            s.bulk_generate(nm, n, seeds[nm])
        rng = np.random.default_rng(55)
        coll = [names[i % 3] for i in range(nreq)]
        ks = rng.integers(3, 51, size=nreq)
        Q = orc.generate(orc.SEED_QUERY, 5000, nreq, dim) * 1.7  # not unit: cosine preprocess
        replies = [None] * nreq
        start = threading.Barrier(nreq)

        def client(i):
            body = json.dumps({"collection": coll[i], "query": Q[i].tolist(),
                               "top_k": int(ks[i]), "filter": {}}).encode()
            start.wait()
            replies[i] = s.handle("POST", "/search", body)

        th = [threading.Thread(target=client, args=(i,)) for i in range(nreq)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        st = s.stats()
        assert st["requests"] >= nreq and st["engine_calls"] < nreq, st  # batched
        # the query goes over the wire as decimal float32 (main.go:28): the
        # oracle preprocesses exactly those values
        Qw = np.array([json.loads(json.dumps(Q[i].tolist())) for i in range(nreq)], np.float32)
        Qp = orc.preprocess(Qw, cosine=True, bf16=True)
        kmax = 50
        for nm in names:
            idx = [i for i in range(nreq) if coll[i] == nm]
            s64, rr, cc = orc.search_generated(seeds[nm], 0, n, Qp[idx], kmax, True)
            for j, i in enumerate(idx):
                stc, body, _ = replies[i]
                assert stc == 200, body
                res = json.loads(body)
                k = int(ks[i])
                assert res["count"] == k and len(res["results"]) == k
                rows = np.array([[_bulk_row(h["id"]) for h in res["results"]]], np.uint64)
                for h, rw in zip(res["results"][:3], rows[0][:3]):
                    assert s.point_id(nm, int(rw)) == h["id"]
                sc = np.array([[h["score"] for h in res["results"]]])
                cnt = np.array([k], np.uint32)
                resc = orc.rescore_generated(seeds[nm], Qp[i:i + 1], rows, cnt, True)
                _check(orc, sc, rows, cnt, s64[j:j + 1, :k], rr[j:j + 1, :k],
                       np.array([min(k, int(cc[j]))], np.uint32), resc, 1e-5)
    finally:
        s.close()
        eng.close()
