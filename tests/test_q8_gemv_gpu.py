"""Single query on the int8 copy (r05; DESIGN.md §5 "Single query on the int8
copy", vs_kernels.hip gemv_q8_*): a one-query search of a collection that
keeps an int8 copy streams the int8 rows (D bytes per row instead of 2D / 4D),
brackets every row's score, and rescores the rows whose upper bound reaches a
lower bound on the k-th score on the GEMV's own per-row arithmetic. The keys
must equal the plain GEMV's bit for bit (an engine opened with
VS_FLAG_NO_PREFILTER keeps no int8 copy and runs the GEMV), and both must pass
the oracle.

Bar (BASELINE.json north_star, oracle.check_topk): rows equal the oracle's
except exact-score near-ties < 1e-5 relative; scores within 1e-5 relative.
Anchor: Points.Search, rag/vector-service/main.go:249-254 (one query, Limit
= top_k); the caller is retrieval-service's searchVectorDB
(rag/retrieval-service/main.go:219-276), one query per request.
"""
import numpy as np
import pytest

SCORE_RTOL = 1e-5


def _same(a, b):
    s1, r1, c1 = a
    s2, r2, c2 = b
    assert np.array_equal(c1, c2)
    assert np.array_equal(r1, r2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))


def _parity(orc, X, Qp, res, k):
    s, r, c = res
    _, s64, rows, cnt = orc.search(X, Qp, k)
    bad = orc.check_topk(s, r, c, s64, rows, cnt, orc.rescore(X, Qp, r, c), SCORE_RTOL)
    assert not bad, bad[:8]


def _one_by_one(e, name, Q, k):
    """Single-query searches (the path under test), stacked."""
    out = [e.search(name, Q[i:i + 1], k) for i in range(Q.shape[0])]
    return tuple(np.concatenate([o[j] for o in out]) for j in range(3))


@pytest.fixture(scope="module")
def c2_pair(pkg):
    """Config C2's corpus: 1M x 768 fp32 cosine, on two engines (int8 copy
    on / off)."""
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    n = 1_000_000
    for e in (a, b):
        e.create_collection("c2", 768, pkg.METRIC_COSINE, pkg.DTYPE_F32, n)
        e.generate("c2", n, 0x5EED)
    assert a.prefilter_bytes("c2") > 0 and b.prefilter_bytes("c2") == 0
    yield a, b, n
    a.close()
    b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [10, 100, 1, 64, 65, 128])
def test_c2_full_size_equals_gemv_and_oracle(c2_pair, orc, k):
    a, b, n = c2_pair
    Q = orc.generate(orc.SEED_QUERY, 0, 4, 768)
    ra = _one_by_one(a, "c2", Q, k)
    rb = _one_by_one(b, "c2", Q, k)
    _same(ra, rb)
    if k in (10, 100):  # the oracle over the full 1M rows (the config's own size)
        X = orc.generate(0x5EED, 0, n, 768)
        _parity(orc, X, orc.preprocess(Q, True, False), ra, k)


@pytest.mark.gpu
def test_c3_corpus_b1_equals_gemv(pkg, orc):
    """10M x 768 bf16 (config C3's corpus, one query): keys equal the GEMV's;
    two queries checked against the streaming fp64 oracle over all rows."""
    n = 10_000_000
    a = pkg.VectorEngine(device=0)
    try:
        a.create_collection("c3", 768, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
        a.generate("c3", n, 0x5EED)
        assert a.prefilter_bytes("c3") > 0
        Q = orc.generate(orc.SEED_QUERY, 1000, 2, 768)
        ra = _one_by_one(a, "c3", Q, 10)
        Qp = orc.preprocess(Q, False, True)
        s64, rr, cc = orc.search_generated(0x5EED, 0, n, Qp, 10, True)
        resc = orc.rescore_generated(0x5EED, Qp, ra[1], ra[2], True)
        bad = orc.check_topk(ra[0], ra[1], ra[2], s64, rr, cc, resc, score_rtol=SCORE_RTOL)
        assert not bad, bad[:4]
    finally:
        a.close()
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        b.create_collection("c3", 768, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
        b.generate("c3", n, 0x5EED)
        _same(ra, _one_by_one(b, "c3", Q, 10))
    finally:
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("dim,dtype,metric", [(1024, "bf16", "cosine"), (768, "bf16", "dot"),
                                              (1024, "f32", "dot")])
def test_shapes_equal_gemv(pkg, orc, dim, dtype, metric):
    dt = pkg.DTYPE_BF16 if dtype == "bf16" else pkg.DTYPE_F32
    mt = pkg.METRIC_COSINE if metric == "cosine" else pkg.METRIC_DOT
    n = 300_000
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        for e in (a, b):
            e.create_collection("s", dim, mt, dt, n)
            e.generate("s", n, 23)
        if dtype == "f32" and dim == 1024:
            # no int8 copy of fp32 1024-d rows (q8_supported): both run the GEMV
            assert a.prefilter_bytes("s") == 0
        else:
            assert a.prefilter_bytes("s") > 0
        Q = orc.generate(orc.SEED_QUERY, 77, 5, dim)
        for k in (5, 50, 128):
            ra = _one_by_one(a, "s", Q, k)
            _same(ra, _one_by_one(b, "s", Q, k))
        X = orc.generate(23, 0, n, dim, bf16=dtype == "bf16")
        _parity(orc, X, orc.preprocess(Q, metric == "cosine", dtype == "bf16"), ra, 128)
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_equal_rows_and_zero_query(pkg, orc):
    """Adversarial brackets: 60k equal rows (every list of their workgroups
    overflows with keys whose U reaches the bound -> those workgroups' rows
    are all rescored) and a zero query (every U equal)."""
    n, dim = 200_000, 768
    X = orc.generate(31, 0, n, dim, bf16=True)
    X[50_000:110_000] = X[7]
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        for e in (a, b):
            e.create_collection("g", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
            e.upsert("g", np.arange(n), X)
        assert a.prefilter_bytes("g") > 0
        Q = orc.generate(orc.SEED_QUERY, 900, 4, dim)
        Q[0] = 0.0
        Q[1] = X[7] * 2.0  # the equal rows lead: ties broken by the lower row
        for k in (10, 100):
            ra = _one_by_one(a, "g", Q, k)
            _same(ra, _one_by_one(b, "g", Q, k))
            _parity(orc, X, orc.preprocess(Q, False, True), ra, k)
        assert list(ra[1][1][:3]) == [7, 50_000, 50_001]
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("density", [0.5, 0.2])
def test_filtered_single_query_equals_gemv(pkg, orc, density):
    """A shipped pre-mask dense enough for the streamed scan (> 1/8 of the
    rows): the int8 scan skips masked rows; keys equal the GEMV's."""
    n, dim = 300_000, 768
    rng = np.random.default_rng(int(density * 100))
    allow = rng.random(n) < density
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        for e in (a, b):
            e.create_collection("f", dim, pkg.METRIC_COSINE, pkg.DTYPE_F32, n)
            e.generate("f", n, 5)
        Q = orc.generate(orc.SEED_QUERY, 4242, 3, dim)
        for i in range(3):
            ra = a.search_filtered("f", Q[i:i + 1], 20, allow)
            rb = b.search_filtered("f", Q[i:i + 1], 20, allow)
            _same(ra, rb)
            assert np.all(allow[ra[1][0][:ra[2][0]]])
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
def test_device_pointer_path_equals_host_path(pkg, orc):
    """vs_search_keys (the bench / shard path, keys on the device) and the
    host path (mapped completion word) give the same keys."""
    import torch
    n, dim, k = 500_000, 768, 10
    e = pkg.VectorEngine(device=0)
    try:
        e.create_collection("d", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
        e.generate("d", n, 99)
        Q = orc.generate(orc.SEED_QUERY, 5, 3, dim)
        for i in range(3):
            s, r, c = e.search("d", Q[i:i + 1], k)
            q = torch.from_numpy(Q[i:i + 1]).cuda()
            keys = torch.zeros((1, k), dtype=torch.int64, device="cuda")
            e.search_keys("d", q.data_ptr(), 1, dim, k, keys.data_ptr(),
                          torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            s2, r2, c2 = pkg.keys_decode(keys.cpu().numpy().view(np.uint64))
            assert np.array_equal(r2, r) and np.array_equal(s2.view(np.uint32), s.view(np.uint32))
    finally:
        e.close()
