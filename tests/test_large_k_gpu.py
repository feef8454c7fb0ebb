"""Searches with k > 128 (the large-k path from k = 129: score pass + device
radix select + sort, vs_select.hip; k > 1024 has no other path), checked
against the oracle on the device.

The reference passes `Limit: uint64(req.TopK)` straight to Qdrant
(rag/vector-service/main.go:249-254), which serves any limit and returns
min(limit, points) hits. Bar as everywhere (BASELINE.json north_star): rows
equal the oracle's up to exact-score near-ties, scores within 1e-5 relative.
Covered: fp32 / bf16, cosine / dot, table and generic dims, k just past the
list limit, k far past it, k above the row count, single queries and
batches, exact ties at the threshold (the row-word digits of the select),
filters (dense, selective, resident, fewer allowed rows than k), a row_base,
a sharded engine, vs_merge_keys at large k, the /search handler at 20k and
1M rows, and the first 128 of a large-k answer equal to the k = 128 list
path's answer bit for bit (the same per-row arithmetic).
"""
import json

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

RTOL = 1e-5


def _parity(orc, X, Qp, s, r, c, k, row_base=0):
    _, s64, rows, cnt = orc.search(X, Qp, k, row_base)
    resc = orc.rescore(X, Qp, r, c, row_base)
    bad = orc.check_topk(s, r, c, s64, rows, cnt, resc, RTOL)
    assert not bad, bad[:10]


@pytest.fixture(scope="module")
def lk_corpora(engine, orc):
    out = {}
    n, dim = 20000, 768
    for dtype in (0, 1):
        for metric in (0, 1):
            name = f"lk_{dtype}_{metric}"
            engine.create_collection(name, dim, metric, dtype)
            engine.generate(name, n, orc.SEED_CORPUS)
            out[(dtype, metric)] = (name, orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=bool(dtype)))
    return out


@pytest.mark.parametrize("k", [129, 700, 1025, 2000, 5000, 20000, 25000])
@pytest.mark.parametrize("dtype,metric", [(0, 0), (1, 0), (1, 1), (0, 1)])
def test_large_k_single_and_batched(engine, orc, lk_corpora, dtype, metric, k):
    name, X = lk_corpora[(dtype, metric)]
    Q = orc.generate(orc.SEED_QUERY, 40, 3, 768) * 1.7
    Qp = orc.preprocess(Q, metric == 0, bool(dtype))
    s, r, c = engine.search(name, Q[:1], k)
    assert int(c[0]) == min(k, X.shape[0])
    _parity(orc, X, Qp[:1], s, r, c, k)
    if k in (2000, 25000):
        s, r, c = engine.search(name, Q, k)  # a batch: one score pass + select per query
        _parity(orc, X, Qp, s, r, c, k)


@pytest.mark.parametrize("dtype", [0, 1])
def test_large_k_prefix_equals_list_path(engine, orc, lk_corpora, dtype):
    """The first 128 keys of a large-k answer (k = 129: the large-k path from
    there, vs_engine.cpp large_k_from; and k = 3000) are the k = 128 list
    path's answer, bit for bit: the score pass forms every row's sum as the
    list scan does."""
    name, _ = lk_corpora[(dtype, 0)]
    Q = orc.generate(orc.SEED_QUERY, 90, 2, 768)
    for i in range(2):
        s1, r1, _ = engine.search(name, Q[i], 128)
        for kk in (129, 3000):
            s3, r3, _ = engine.search(name, Q[i], kk)
            assert np.array_equal(r3[:, :128], r1)
            assert np.array_equal(s3[:, :128].view(np.uint32), s1.view(np.uint32))


@pytest.mark.parametrize("dim,dtype", [(128, 0), (1536, 1), (100, 1), (100, 0)])
def test_large_k_dims(pkg, orc, dim, dtype):
    with pkg.VectorEngine(device=0) as eng:
        n = 6000
        eng.create_collection("d", dim, 0, dtype)
        eng.generate("d", n, orc.SEED_CORPUS)
        X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=bool(dtype))
        Q = orc.generate(orc.SEED_QUERY, 7, 2, dim)
        s, r, c = eng.search("d", Q, 1500)
        _parity(orc, X, orc.preprocess(Q, True, bool(dtype)), s, r, c, 1500)


def test_large_k_exact_ties(pkg, orc):
    """Many rows with identical scores straddle the k-th position: the select
    walks the row word (lower rows first), and rows beyond it are dropped."""
    dim = 256
    rng = np.random.default_rng(3)
    base = orc.generate(11, 0, 7, dim)
    idx = rng.integers(0, 7, size=9000)
    V = base[idx]
    V[::97] = orc.generate(12, 0, V[::97].shape[0], dim)  # some distinct rows too
    with pkg.VectorEngine(device=0) as eng:
        for dtype in (0, 1):
            eng.create_collection(f"t{dtype}", dim, 1, dtype, 0, 77)  # dot, row_base 77
            eng.upsert(f"t{dtype}", np.arange(V.shape[0]), V)
            X = orc.preprocess(V, False, bool(dtype))
            Q = base[:3] + 0.01 * orc.generate(13, 0, 3, dim)
            Qp = orc.preprocess(Q, False, bool(dtype))
            for k in (1100, 2500, 4321, 8999):
                s, r, c = eng.search(f"t{dtype}", Q, k)
                _parity(orc, X, Qp, s, r, c, k, row_base=77)
                # within a run of equal scores the rows ascend (the tie rule)
                for i in range(3):
                    eq = np.diff(s[i, :int(c[i])]) == 0
                    assert np.all(np.diff(r[i, :int(c[i])].astype(np.int64))[eq] > 0)


@pytest.mark.parametrize("density", [0.5, 0.02, 0.0005])
def test_large_k_filtered(engine, orc, lk_corpora, density):
    name, X = lk_corpora[(1, 0)]
    n = X.shape[0]
    rng = np.random.default_rng(int(density * 1e4))
    allow = rng.random(n) < density
    Q = orc.generate(orc.SEED_QUERY, 500, 2, 768)
    Qp = orc.preprocess(Q, True, True)
    Xm = X[allow]
    rows_allowed = np.nonzero(allow)[0]
    fid = engine.filter_create(name, allow)
    try:
        for k in (1100, 3000):
            for how in ("bitmap", "resident"):
                if how == "bitmap":
                    s, r, c = engine.search_filtered(name, Q, k, allow)
                else:
                    s, r, c = engine.search_filter_id(name, Q, k, fid)
                assert np.all(c == min(k, int(allow.sum())))
                # oracle over the allowed rows only, rows mapped back
                _, s64, rr, cc = orc.search(Xm, Qp, k)
                rr = np.where(np.arange(rr.shape[1])[None, :] < cc[:, None],
                              rows_allowed[np.minimum(rr, len(rows_allowed) - 1)], 0)
                resc = orc.rescore(X, Qp, r, c)
                bad = orc.check_topk(s, r, c, s64, rr, cc, resc, RTOL)
                assert not bad, (k, how, bad[:5])
                assert np.all(allow[r[0, :int(c[0])].astype(np.int64)])
    finally:
        engine.filter_drop(fid)


def test_large_k_sharded_equals_single(pkg, orc):
    """A 3-shard engine (row stripes on device 0) merges the shards' k-key
    lists with the sort merge: equal to one device."""
    dim, n = 384, 30000
    with pkg.VectorEngine(device=0) as one, pkg.VectorEngine(shards=[0, 0, 0]) as sh:
        for e in (one, sh):
            e.create_collection("s", dim, 0, 1)
            e.generate("s", n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 3, 3, dim)
        for k in (1500, 4000):
            a = one.search("s", Q, k)
            b = sh.search("s", Q, k)
            assert np.array_equal(a[1], b[1]) and np.array_equal(a[0], b[0]) and np.array_equal(a[2], b[2])
        X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
        s, r, c = sh.search("s", Q, 4000)
        _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, 4000)


@pytest.mark.timeout(600)
def test_large_k_1m_rows(engine, orc, pkg):
    n, dim = 1_000_000, 768
    name = "lk1m"
    engine.create_collection(name, dim, pkg.METRIC_COSINE, pkg.DTYPE_F32, n)
    try:
        engine.generate(name, n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 77, 2, dim)
        Qp = orc.preprocess(Q, cosine=True, bf16=False)
        for k in (2000, 5000):
            s, r, c = engine.search(name, Q, k)
            s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp, k, False)
            resc = orc.rescore_generated(orc.SEED_CORPUS, Qp, r, c, False)
            bad = orc.check_topk(s, r, c, s64, rr, cc, resc, RTOL)
            assert not bad, bad[:5]
    finally:
        engine.drop_collection(name)


def _bulk_row(uuid: str) -> int:
    return int(uuid.replace("-", ""), 16) & ((1 << 62) - 1)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("n", [20_000, 1_000_000])
def test_search_handler_large_top_k(pkg, orc, n):
    """/search with top_k 2000 and 5000: 200, count = top_k, the oracle's rows."""
    from importlib import import_module
    svcmod = import_module(pkg.__name__ + ".service")
    dim = 768
    cfg = {"collections": [{"name": "regulatory_docs", "dim": dim, "metric": "Cosine",
                            "dtype": "f32"}]}
    eng = pkg.VectorEngine(device=0)
    s = svcmod.VectorService(eng, cfg)
    try:
        s.bulk_generate("regulatory_docs", n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 901, 2, dim) * 0.3
        Qw = np.array([json.loads(json.dumps(Q[i].tolist())) for i in range(2)], np.float32)
        Qp = orc.preprocess(Qw, cosine=True, bf16=False)
        for k in (2000, 5000):
            s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp, k, False)
            for i in range(2):
                body = json.dumps({"collection": "regulatory_docs", "query": Q[i].tolist(),
                                   "top_k": k, "filter": None}).encode()
                st, out, _ = s.handle("POST", "/search", body)
                assert st == 200, out[:300]
                res = json.loads(out)
                assert res["count"] == k and len(res["results"]) == k
                rows = np.array([[_bulk_row(h["id"]) for h in res["results"]]], np.uint64)
                sc = np.array([[h["score"] for h in res["results"]]])
                cnt = np.array([k], np.uint32)
                resc = orc.rescore_generated(orc.SEED_CORPUS, Qp[i:i + 1], rows, cnt, False)
                bad = orc.check_topk(sc, rows, cnt, s64[i:i + 1], rr[i:i + 1], cc[i:i + 1], resc, RTOL)
                assert not bad, (n, k, bad[:5])
        # top_k past the row count: every point, Qdrant's min(limit, points)
        if n == 20_000:
            body = json.dumps({"collection": "regulatory_docs", "query": Q[0].tolist(),
                               "top_k": 1 << 40}).encode()
            st, out, _ = s.handle("POST", "/search", body)
            assert st == 200 and json.loads(out)["count"] == n
    finally:
        s.close()
        eng.close()


_RSEL_AB = r"""
import json, sys
import torch                      # first: the library then binds torch's HIP runtime
import numpy as np
sys.path.insert(0, ROOT)
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
out = {}
with pkg.VectorEngine(device=0) as eng:
    eng.create_collection("r", 768, 1, 1, 0, 5)
    eng.generate("r", 200_000, orc.SEED_CORPUS)
    Q = orc.generate(orc.SEED_QUERY, 0, 3, 768)
    for k in (129, 4000, 5000, 50_000):
        s, r, c = eng.search("r", Q, k)
        out[f"r/{k}"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
    # identical rows: the boundary bucket holds thousands of equal scores
    base = orc.generate(11, 0, 5, 256)
    V = base[np.arange(30_000) % 5]
    eng.create_collection("t", 256, 1, 0, 0, 9)
    eng.upsert("t", np.arange(V.shape[0]), V)
    for k in (3000, 12_345, 29_999):
        s, r, c = eng.search("t", base[:2] + 0.001, k)
        out[f"t/{k}"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
print(json.dumps(out))
"""


def test_fused_selection_equals_digit_chain():
    """The one-launch selection (rsel_fused_kernel: first digit from the score
    pass's histogram, one compaction pass, the last workgroup finishing the
    boundary bucket by an LDS sort or radix passes) must return the same bits
    as the 12-launch digit chain (VS_RSEL_FUSED=0): random rows at k = 129 ..
    50,000 and 30,000 rows of 5 repeated vectors (ties across the k-th key)."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

    def run(env_extra):
        env = dict(os.environ, **env_extra)
        res = subprocess.run([sys.executable, "-c", f"ROOT={root!r}\n" + _RSEL_AB],
                             capture_output=True, text=True, timeout=300, env=env)
        assert res.returncode == 0, res.stderr[-3000:]
        return json.loads(res.stdout.strip().splitlines()[-1])

    a = run({})
    b = run({"VS_RSEL_FUSED": "0"})
    assert a.keys() == b.keys()
    bad = [key for key in a if a[key] != b[key]]
    assert not bad, bad
