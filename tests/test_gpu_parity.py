"""Device parity against the oracle, through the C-ABI (run on an MI355X).

Bar (BASELINE.json north_star): returned rows equal the oracle's except for
near-ties (< 1e-5 relative), scores within 1e-5 relative of the exact score
(the spec allows 2e-3 for bf16; the tests hold bf16 to 1e-5 as well, because
the oracle scores the same bf16 values). Stored rows and generated corpora
are compared bit for bit.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCORE_RTOL = 1e-5


def _parity(orc, X, Qp, s, r, c, k, row_base=0):
    s32, s64, rows, cnt = orc.search(X, Qp, k, row_base)
    resc = orc.rescore(X, Qp, r, c, row_base)
    bad = orc.check_topk(s, r, c, s64, rows, cnt, resc, SCORE_RTOL)
    assert not bad, bad[:10]
    return rows


# ------------------------------------------------------------- store side
@pytest.mark.parametrize("dtype", [0, 1])
@pytest.mark.parametrize("dim", [768, 1024, 100])
def test_generate_bit_exact(engine, orc, dtype, dim):
    name = f"gen_{dtype}_{dim}"
    engine.create_collection(name, dim, 0, dtype)
    engine.generate(name, 3000, orc.SEED_CORPUS)
    engine.generate(name, 1000, orc.SEED_CORPUS)  # appended rows continue the row numbers
    got = engine.read_rows(name, 0, 4000)
    ref = orc.generate(orc.SEED_CORPUS, 0, 4000, dim, bf16=bool(dtype))
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    engine.drop_collection(name)


@pytest.mark.parametrize("metric", [0, 1])
@pytest.mark.parametrize("dtype", [0, 1])
def test_upsert_preprocess_bit_exact(engine, orc, metric, dtype):
    rng = np.random.default_rng(11)
    dim = 768
    raw = (rng.standard_normal((300, dim)) * rng.uniform(1e-3, 1e3, (300, 1))).astype(np.float32)
    raw[0] = 0
    raw[1] = orc.generate(orc.SEED_QUERY, 0, 1, dim)[0]
    name = f"ups_{metric}_{dtype}"
    engine.create_collection(name, dim, metric, dtype)
    engine.upsert(name, np.arange(300), raw)
    got = engine.read_rows(name, 0, 300)
    ref = orc.preprocess(raw, metric == 0, bool(dtype))
    assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    engine.drop_collection(name)


def test_upsert_overwrite_and_duplicates(engine, orc):
    dim = 64
    engine.create_collection("ow", dim, 0, 0)
    a = orc.generate(1, 0, 10, dim)
    engine.upsert("ow", np.arange(10), a)
    b = orc.generate(2, 0, 3, dim)
    # overwrite rows 2 and 7; append 10; duplicate row 7: last occurrence wins
    engine.upsert("ow", [2, 7, 10, 7], np.stack([b[0], b[1], b[2], a[0]]))
    got = engine.read_rows("ow", 0, 11)
    exp = np.concatenate([a, b[2:3]])
    exp[2] = b[0]
    exp[7] = a[0]
    assert np.array_equal(got, orc.preprocess(exp, True))
    assert engine.collection_info("ow")["rows"] == 11
    with pytest.raises(Exception):
        engine.upsert("ow", [13], a[:1])  # hole
    with pytest.raises(Exception):
        engine.upsert("ow", [0], np.zeros((1, dim + 1), np.float32))  # dim mismatch
    engine.drop_collection("ow")


def test_upsert_chunked_staging_bit_exact(engine, orc):
    """Upserts larger than one 16 MiB staging chunk, through both pinned buffers:
    an ascending append (the copy-through path), then a shuffled overwrite with
    duplicates (the sorted path, last occurrence wins), then a small append after
    the staging has grown — every stored row bit-exact with the oracle's
    preprocess (rag/vector-service/main.go:165-182 → Qdrant upsert)."""
    rng = np.random.default_rng(21)
    dim, n = 256, 100_000  # 16 MiB / (1 KiB + 8 B) = 16,256 rows per chunk: 7 chunks
    engine.create_collection("chunked", dim, 0, 1)
    try:
        X = (rng.standard_normal((n, dim)) * rng.uniform(0.1, 10, (n, 1))).astype(np.float32)
        engine.upsert("chunked", np.arange(n, dtype=np.uint64), X)
        ids = rng.integers(0, n, 70_000).astype(np.uint64)  # duplicates included
        Y = rng.standard_normal((len(ids), dim)).astype(np.float32)
        engine.upsert("chunked", ids, Y)
        exp = X.copy()
        u, first = np.unique(ids[::-1], return_index=True)
        exp[u] = Y[len(ids) - 1 - first]  # the last occurrence of each row wins
        Z = rng.standard_normal((5, dim)).astype(np.float32)
        engine.upsert("chunked", np.arange(n, n + 5), Z)
        exp = np.concatenate([exp, Z])
        got = engine.read_rows("chunked", 0, n + 5)
        ref = orc.preprocess(exp, True, True)
        assert np.array_equal(got.view(np.uint32), ref.view(np.uint32))
    finally:
        engine.drop_collection("chunked")


# ------------------------------------------------------------- search side
@pytest.fixture(scope="module")
def corpora(engine, orc):
    """1 x fp32 and 1 x bf16 collection of 20k x 768 synthetic rows."""
    out = {}
    n, dim = 20000, 768
    for dtype in (0, 1):
        name = f"c768_{dtype}"
        engine.create_collection(name, dim, 0, dtype)
        engine.generate(name, n, orc.SEED_CORPUS)
        out[dtype] = (name, orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=bool(dtype)))
    return out


@pytest.mark.parametrize("k", [1, 5, 10, 64, 100, 1024])
@pytest.mark.parametrize("dtype", [0, 1])
def test_gemv_single_query(engine, orc, corpora, dtype, k):
    name, X = corpora[dtype]
    Q = orc.generate(orc.SEED_QUERY, 0, 3, 768)
    for i in range(3):
        s, r, c = engine.search(name, Q[i], k)
        _parity(orc, X, orc.preprocess(Q[i:i + 1], True, bool(dtype)), s, r, c, k)


@pytest.mark.parametrize("nq,k", [(2, 10), (33, 1), (256, 10), (300, 16), (64, 5)])
def test_mfma_batched(engine, orc, corpora, nq, k):
    name, X = corpora[1]
    Q = orc.generate(orc.SEED_QUERY, 100, nq, 768)
    s, r, c = engine.search(name, Q, k)
    _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k)


@pytest.fixture(scope="module")
def corpus_fast(engine, orc):
    """200k x 768 bf16: >= 8 tiles per workgroup, so batched searches take the
    sample pass + candidate-buffer main pass (vs_engine.cpp search_core)."""
    n, dim = 200_000, 768
    engine.create_collection("fast768", dim, 0, 1, n)
    engine.generate("fast768", n, orc.SEED_CORPUS)
    return "fast768", orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)


@pytest.mark.parametrize("nq,k", [(2, 10), (256, 10), (300, 16), (77, 1), (256, 5), (256, 17),
                                  (64, 50), (300, 100), (33, 128)])
def test_mfma_candidate_path(engine, orc, corpus_fast, nq, k):
    name, X = corpus_fast
    Q = orc.generate(orc.SEED_QUERY, 1000, nq, 768)
    s, r, c = engine.search(name, Q, k)
    _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k)


@pytest.mark.parametrize("dim,nq,k", [(1024, 200, 10), (1536, 129, 50), (128, 256, 10),
                                      (512, 300, 5)])
def test_mfma_candidate_path_dims(engine, orc, dim, nq, k):
    """Candidate path at other dims: 1024 / 1536 run 128 queries per launch."""
    n = 100_000
    name = f"fast{dim}"
    engine.create_collection(name, dim, 0, 1, n)
    engine.generate(name, n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 3000, nq, dim)
    s, r, c = engine.search(name, Q, k)
    _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k)
    engine.drop_collection(name)


def test_mfma_full_quarter_replacement(engine, orc):
    """Adversarial ties: 300k rows, the first 200k identical. Every identical
    row reaches the sample bound of the queries that match it, so every lane
    of those queries appends a slab per tile (~24 per workgroup) and its
    quarter of the candidate buffer fills; the main pass then keeps the best
    slabs in place (ties -> the earlier tile) and must still give the exact
    answer (ties -> lowest rows) for those queries and for the others alike,
    with no re-run, at every k the quarter size covers."""
    n, dim = 300_000, 768
    base = orc.generate(orc.SEED_CORPUS, 0, n, dim)
    base[:200_000] = base[12_345]
    engine.create_collection("ties", dim, 0, 1, n)
    engine.upsert("ties", np.arange(n), base)
    X = orc.preprocess(base, True, True)
    Q = np.concatenate([base[12_345:12_346], orc.generate(orc.SEED_QUERY, 7, 40, dim),
                        base[12_345:12_346] * 3.0])
    for k in (1, 10, 16, 50, 128):
        s, r, c = engine.search("ties", Q, k)
        assert r[0].tolist() == list(range(k)) and r[-1].tolist() == list(range(k))
        _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k)
    engine.drop_collection("ties")


def test_mfma_select_spill_ties(engine, orc):
    """70k rows, the first 40k identical: each workgroup's ~9 tiles fit its
    16-slab quarters (no overflow), but ~40k keys tie at the top for the
    matching queries, so the select streams the slabs in chunks (its spill
    path) and must still return the lowest rows."""
    n, dim = 70_000, 768
    base = orc.generate(orc.SEED_CORPUS, 0, n, dim)
    base[:40_000] = base[12_345]
    engine.create_collection("ties70", dim, 0, 1, n)
    engine.upsert("ties70", np.arange(n), base)
    X = orc.preprocess(base, True, True)
    Q = np.concatenate([base[12_345:12_346], orc.generate(orc.SEED_QUERY, 9, 40, dim)])
    for k in (10, 50, 128):
        s, r, c = engine.search("ties70", Q, k)
        assert r[0].tolist() == list(range(k))
        _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k)
    engine.drop_collection("ties70")


def test_fp32_batched(engine, orc, corpora):
    name, X = corpora[0]
    Q = orc.generate(orc.SEED_QUERY, 500, 5, 768)
    s, r, c = engine.search(name, Q, 10)
    _parity(orc, X, orc.preprocess(Q, True, False), s, r, c, 10)


def test_golden_fixture_on_device(engine, orc):
    import os
    g = np.load(os.path.join(os.path.dirname(__file__), "golden", "search_4096x768.npz"))
    Q = orc.generate(orc.SEED_QUERY, 0, 32, 768)
    for tag, dtype in (("f32", 0), ("bf16", 1)):
        name = f"gold_{tag}"
        engine.create_collection(name, 768, 0, dtype)
        engine.generate(name, 4096, orc.SEED_CORPUS)
        X = orc.generate(orc.SEED_CORPUS, 0, 4096, 768, bf16=bool(dtype))
        for k in (1, 5, 10, 100):
            s, r, c = engine.search(name, Q, k)
            resc = orc.rescore(X, g[f"qpre_{tag}"], r, c)
            bad = orc.check_topk(s, r, c, g[f"scores64_{tag}_k{k}"], g[f"rows_{tag}_k{k}"],
                                 np.full(32, k, np.uint32), resc, SCORE_RTOL)
            assert not bad, (tag, k, bad[:5])
        engine.drop_collection(name)


@pytest.mark.parametrize("dim", [100, 384, 1024, 1536, 256, 128, 512])
@pytest.mark.parametrize("dtype", [0, 1])
def test_other_dims(engine, orc, dim, dtype):
    n = 3001
    name = f"d{dim}_{dtype}"
    engine.create_collection(name, dim, 0, dtype)
    engine.generate(name, n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=bool(dtype))
    Q = orc.generate(orc.SEED_QUERY, 0, 6, dim)
    for nq in (1, 6):
        s, r, c = engine.search(name, Q[:nq], 7)
        _parity(orc, X, orc.preprocess(Q[:nq], True, bool(dtype)), s, r, c, 7)
    engine.drop_collection(name)


# ------------------------------------------------------------- edge cases
@pytest.mark.parametrize("dtype", [0, 1])
def test_edges(engine, orc, dtype):
    dim = 768
    name = f"edge_{dtype}"
    engine.create_collection(name, dim, 0, dtype)
    q = orc.generate(orc.SEED_QUERY, 0, 2, dim)
    # empty collection -> no results
    s, r, c = engine.search(name, q, 5)
    assert c.tolist() == [0, 0]
    base = orc.generate(orc.SEED_CORPUS, 0, 7, dim)
    vecs = np.concatenate([base, base[[3, 3]], np.zeros((1, dim), np.float32)])  # dups + zero row
    engine.upsert(name, np.arange(10), vecs)
    X = orc.preprocess(vecs, True, bool(dtype))
    # k > rows
    s, r, c = engine.search(name, q, 50)
    assert c.tolist() == [10, 10]
    _parity(orc, X, orc.preprocess(q, True, bool(dtype)), s, r, c, 50)
    # exact duplicates tie -> row ascending; self match first
    s, r, c = engine.search(name, base[[3, 3]], 3)
    assert r[0].tolist() == [3, 7, 8] and r[1].tolist() == [3, 7, 8]
    # zero query: every score 0, rows ascending
    s, r, c = engine.search(name, np.zeros((1, dim), np.float32), 4)
    assert r[0].tolist() == [0, 1, 2, 3] and np.all(s == 0)
    with pytest.raises(Exception):
        engine.search(name, np.zeros((1, dim - 1), np.float32), 4)
    with pytest.raises(Exception):
        engine.search(name, q, 0)
    with pytest.raises(Exception):
        engine.search("nope", q, 3)
    engine.drop_collection(name)


def test_dot_metric(engine, orc):
    dim = 768
    rng = np.random.default_rng(5)
    X = (rng.standard_normal((5000, dim)) * rng.uniform(0.1, 3, (5000, 1))).astype(np.float32)
    q = rng.standard_normal((3, dim)).astype(np.float32)
    for dtype in (0, 1):
        name = f"dot_{dtype}"
        engine.create_collection(name, dim, 1, dtype)
        engine.upsert(name, np.arange(5000), X)
        Xs = orc.preprocess(X, False, bool(dtype))
        for nq in (1, 3):
            s, r, c = engine.search(name, q[:nq], 10)
            _parity(orc, Xs, orc.preprocess(q[:nq], False, bool(dtype)), s, r, c, 10)
        engine.drop_collection(name)


# ----------------------------------------------- sharded merge on one device
_SHARDED = r"""
import sys, json
import torch                      # first: the library then binds torch's HIP runtime
import numpy as np
sys.path.insert(0, ROOT)
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
eng = pkg.VectorEngine(device=0)
dim, n, P, nq, k = 768, 30000, 4, 40, 10
per = (n + P - 1) // P
for p in range(P):
    lo, hi = p * per, min(n, (p + 1) * per)
    eng.create_collection(f"shard{p}", dim, 0, 1, 0, lo)
    eng.generate(f"shard{p}", hi - lo, orc.SEED_CORPUS)
dq = torch.empty((nq, dim), dtype=torch.float32, device="cuda")
st = torch.cuda.current_stream().cuda_stream
eng.generate_vectors(orc.SEED_QUERY, 0, nq, dim, dq.data_ptr(), st)
lists = torch.zeros((P, nq, k), dtype=torch.int64, device="cuda")
for p in range(P):
    eng.search_keys(f"shard{p}", dq.data_ptr(), nq, dim, k, lists[p].data_ptr(), st)
out = torch.zeros((nq, k), dtype=torch.int64, device="cuda")
eng.merge_keys(lists.data_ptr(), P, nq, k, k, out.data_ptr(), st)
s, r, c = eng.decode_keys(out.data_ptr(), nq, k, st)
# the device-generated queries equal the oracle's generator rows
assert np.array_equal(dq.cpu().numpy(), orc.generate(orc.SEED_QUERY, 0, nq, dim))
X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
Qp = orc.preprocess(orc.generate(orc.SEED_QUERY, 0, nq, dim), True, True)
s32, s64, rows, cnt = orc.search(X, Qp, k)
resc = orc.rescore(X, Qp, r, c)
bad = orc.check_topk(s, r, c, s64, rows, cnt, resc, 1e-5)
print(json.dumps({"bad": bad[:10]}))
"""


def _run_py(code, timeout=300):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    res = subprocess.run([sys.executable, "-c", f"ROOT={root!r}\n" + code], capture_output=True,
                         text=True, timeout=timeout)
    assert res.returncode == 0, res.stderr[-3000:]
    return json.loads(res.stdout.strip().splitlines()[-1])


def test_sharded_merge_equals_unsharded():
    """4 row shards (row_base offsets) searched by device pointer, keys merged on device."""
    assert _run_py(_SHARDED)["bad"] == []


def test_bench_small_runs():
    """bench.py end to end (torch first, device queries, JSON line) on a small corpus."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    for cfg in ("c3", "c2"):
        res = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--config", cfg,
                              "--rows", "300000", "--steps", "3", "--warmup", "1",
                              "--cpu-sample-rows", "20000", "--cpu-budget-s", "0.5"],
                             capture_output=True, text=True, timeout=300)
        assert res.returncode == 0, res.stderr[-3000:]
        line = json.loads(res.stdout.strip().splitlines()[-1])
        assert line["value"] > 0 and line["roofline"]["frac"] > 0
        assert line["cpu_baseline"]["value"] > 0
        assert line["cpu_baseline"]["cpu_model"] and line["cpu_baseline"]["isa"] in ("avx2", "avx512")
        if cfg == "c3":  # batched config: the BLAS secondary is reported too
            assert line["cpu_baseline"]["batched"]["value"] > 0
            assert line["secondary"]["steps_verified"] >= 100
        # r04: every timed step checked after the timer, and the timed batch
        # checked against the oracle over the whole (300k-row) corpus
        assert line["steps_verified"] == 3
        assert line["parity"]["queries_checked"] >= 1 and line["parity"]["violations"] == 0, \
            line["parity"]


def test_large_properties(engine, orc):
    """Size-independent checks at 2M rows: self-match and monotone k-prefixes."""
    dim, n = 768, 2_000_000
    engine.create_collection("big", dim, 0, 1, n)
    engine.generate("big", n, orc.SEED_CORPUS)
    probe = [0, 123457, 1999999]
    Xp = orc.generate(orc.SEED_CORPUS, 0, 1, dim, True)  # noqa: F841 (warm)
    Q = np.concatenate([orc.generate(orc.SEED_CORPUS, i, 1, dim, True) for i in probe])
    s, r, c = engine.search("big", Q, 10)            # MFMA path
    assert r[:, 0].tolist() == probe and np.all(np.abs(s[:, 0] - 1) < 1e-2)
    for i, p in enumerate(probe):
        s1, r1, c1 = engine.search("big", Q[i], 10)  # GEMV path
        assert r1[0, 0] == p
        s2, r2, c2 = engine.search("big", Q[i], 100)
        assert r2[0, :10].tolist() == r1[0].tolist()
        assert np.all(np.diff(s2[0]) <= 0)
    engine.drop_collection("big")


def test_mfma_large_shard_parity_128(engine, orc):
    """Large shard with a partial last tile: full oracle parity at dim 128,
    4.4M + 17 rows (537 tiles per workgroup), 64 queries, repeated; probes
    that are corpus rows from the start, the middle and the partial last
    tile must each be their own top hit."""
    dim, n = 128, 4_400_017
    engine.create_collection("big128", dim, 0, 1, n)
    engine.generate("big128", n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 7, 64, dim)
    for _ in range(2):
        s, r, c = engine.search("big128", Q, 10)
        _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, 10)
    probe = [0, 1_000_003, n * 7 // 8 + 11, n - 40, n - 17, n - 1]
    P = np.stack([X[i] for i in probe] + [X[5]] * 58)
    s, r, c = engine.search("big128", P, 1)
    assert r[:len(probe), 0].tolist() == probe
    engine.drop_collection("big128")


@pytest.mark.parametrize("k", [10, 100])
def test_mfma_parity_1m_768(engine, orc, k):
    """Full oracle parity at dim 768 on 1M + 3 rows (122 tiles per
    workgroup, a partial last tile), 64 queries, k = 10 and 100."""
    dim, n = 768, 1_000_003
    try:
        engine.collection_info("c1m768")
    except Exception:
        engine.create_collection("c1m768", dim, 0, 1, n)
        engine.generate("c1m768", n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 300, 64, dim)
    s, r, c = engine.search("c1m768", Q, k)
    _parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k)
    if k == 100:
        engine.drop_collection("c1m768")


def test_mfma_probes_4_5m_768(engine, orc):
    """4.5M + 5 rows at dim 768: probes across the corpus and in the last
    tile find themselves, and each probe's batched top-10 equals the GEMV
    path's (where no near-tie makes the order ambiguous)."""
    dim, n = 768, 4_500_005
    engine.create_collection("big768", dim, 0, 1, n)
    engine.generate("big768", n, orc.SEED_CORPUS)
    probe = [17, 2_250_001, n * 7 // 8 + 3, n * 15 // 16, n - 5, n - 1]
    Q = np.concatenate([orc.generate(orc.SEED_CORPUS, i, 1, dim, True) for i in probe])
    Qb = np.concatenate([Q] + [orc.generate(orc.SEED_QUERY, 0, 250, dim)])
    s, r, c = engine.search("big768", Qb, 10)  # MFMA path
    assert r[:len(probe), 0].tolist() == probe
    for i, p in enumerate(probe):
        s1, r1, c1 = engine.search("big768", Q[i], 10)  # GEMV path
        assert r1[0, 0] == p
        np.testing.assert_allclose(s[i], s1[0], rtol=1e-5, atol=1e-6)
        if np.abs(np.diff(s1[0])).min() > 1e-5:
            assert r[i].tolist() == r1[0].tolist()
    engine.drop_collection("big768")


def test_health(engine):
    import json
    h = json.loads(engine.health())
    assert h["status"] == "healthy" and h["hbm_total_bytes"] > 0


@pytest.mark.parametrize("sample,expect", [(False, 20), (True, 5)])
def test_scan_timing(orc, sample, expect):
    """VS_FLAG_TIMING brackets every scan; with VS_FLAG_TIMING_SAMPLE one batched
    scan in 4 (the 4th, 8th, ...; one-query scans: one in 16)."""
    import __graft_entry__ as ge
    pkg = ge.load_package()
    with pkg.VectorEngine(device=0, timing=True, timing_sample=sample) as eng:
        eng.create_collection("t", 768, 0, 1, 20_000)
        eng.generate("t", 20_000, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 0, 4, 768)
        for _ in range(20):
            eng.search("t", Q, 10)
        t = eng.timing(reset=True)
        assert t["scan_n"] == expect and t["scan_ms"] > 0


_MERGE_DUP = r"""
import sys, json
sys.path.insert(0, ROOT)
import numpy as np, torch
import __graft_entry__ as ge
pkg = ge.load_package()
eng = pkg.VectorEngine(device=0)
rng = np.random.default_rng(5)
bad = []
# (lists, k_in, k, distinct keys): rank path (<= 512 keys), tournament path
# (<= 8192 keys, k <= 32), general path (k > 32)
# and the sort merge of k or k_in > 1024 (vs_select.hip launch_merge_large)
for L, kin, k, nd in ((8, 10, 10, 6), (8, 10, 64, 30), (40, 100, 20, 15), (40, 100, 20, 300),
                      (12, 100, 100, 50), (12, 100, 100, 700), (100, 100, 100, 2000),
                      (4, 2000, 3000, 5000), (3, 1500, 1500, 2000), (8, 10, 2000, 50),
                      (5, 1200, 1100, 900),
                      # r03 sample bound + list walk (k > 32 or many keys): many
                      # lists, heavy overlap (survivors past the LDS buffer:
                      # the filter fallback), two long lists, kin < k
                      (758, 100, 100, 20000), (758, 100, 100, 400), (1000, 100, 100, 3000),
                      (2, 1024, 1024, 3000), (1500, 16, 100, 8000), (64, 128, 128, 10000),
                      (33, 50, 40, 5000), (5000, 8, 64, 30000)):
    nq = 3
    pool = np.unique(rng.integers(1 << 40, 1 << 62, size=nd * 2, dtype=np.uint64))[:nd]
    lists = np.zeros((L, nq, kin), np.uint64)
    for l in range(L):
        for q in range(nq):
            m = min(kin, int(rng.integers(0, kin + 1)), nd)
            pick = np.sort(rng.choice(pool, size=m, replace=False))[::-1]
            lists[l, q, :m] = pick
    d = torch.from_numpy(lists.view(np.int64)).cuda()
    out = torch.full((nq, k), 12345, dtype=torch.int64, device="cuda")  # poisoned
    st = torch.cuda.current_stream().cuda_stream
    eng.merge_keys(d.data_ptr(), L, nq, kin, k, out.data_ptr(), st)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    for q in range(nq):
        u = np.unique(lists[:, q, :][lists[:, q, :] != 0])[::-1]
        want = np.zeros(k, np.uint64)
        want[:min(k, u.size)] = u[:k]
        if not np.array_equal(got[q], want):
            bad.append([L, kin, k, nd, q, got[q][:8].tolist(), want[:8].tolist()])
# replicated lists (every list the same keys): the sample's ranks count each
# key L times, so its bound overshoots; the merge must notice and fall back
for L, kin, k, nd in ((5000, 64, 100, 64), (600, 100, 100, 100), (40, 100, 64, 70)):
    nq = 2
    one = np.zeros((nq, kin), np.uint64)
    for q in range(nq):
        pool = np.unique(rng.integers(1 << 40, 1 << 62, size=nd * 2, dtype=np.uint64))[:nd]
        one[q, :min(kin, nd)] = np.sort(pool)[::-1][:kin]
    lists = np.ascontiguousarray(np.broadcast_to(one, (L, nq, kin)))
    d = torch.from_numpy(lists.view(np.int64)).cuda()
    out = torch.full((nq, k), 12345, dtype=torch.int64, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    eng.merge_keys(d.data_ptr(), L, nq, kin, k, out.data_ptr(), st)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint64)
    for q in range(nq):
        u = np.unique(one[q][one[q] != 0])[::-1]
        want = np.zeros(k, np.uint64)
        want[:min(k, u.size)] = u[:k]
        if not np.array_equal(got[q], want):
            bad.append(["replicated", L, kin, k, q, got[q][:8].tolist(), want[:8].tolist()])
print(json.dumps({"bad": bad[:5]}))
"""


def test_merge_dedupes_and_zero_fills():
    """vs_merge_keys with keys repeated across lists (overlapping shards), fewer
    distinct keys than k and a poisoned output: each key once, the rest 0, on
    the rank, tournament and general paths and the large-k sort merge."""
    assert _run_py(_MERGE_DUP)["bad"] == []


@pytest.mark.parametrize("dim", [128, 768, 1536])
@pytest.mark.parametrize("dtype", [0, 1])
@pytest.mark.parametrize("metric", [0, 1])
def test_small_collection_one_launch(pkg, orc, dim, dtype, metric):
    """One query over <= 256 rows with k <= 16 takes the one-launch path
    (launch_gemv_small: query prep + scan + merge in one workgroup). Its keys
    must equal the first k of the three-launch path's (k = 17 takes that path),
    bit for bit, and the oracle's top k; rows < k, one row and a row_base too."""
    bf16 = dtype == 1
    rng = np.random.default_rng(dim * 4 + dtype * 2 + metric)
    with pkg.VectorEngine(device=0) as eng:
        for rows, base in ((1, 0), (5, 0), (63, 0), (221, 0), (256, 1000)):
            name = f"s{rows}"
            eng.create_collection(name, dim, metric, dtype, 0, base)
            V = rng.standard_normal((rows, dim)).astype(np.float32)
            eng.upsert(name, list(range(rows)), V)
            X = orc.preprocess(V, metric == 0, bf16)
            for t in range(3):
                Q = (rng.standard_normal((1, dim)) * (1 + 3 * t)).astype(np.float32)
                s17, r17, c17 = eng.search(name, Q, 17)
                Qp = orc.preprocess(Q, metric == 0, bf16)
                for k in (1, 5, 16):
                    s, r, c = eng.search(name, Q, k)
                    assert int(c[0]) == min(rows, k)
                    assert np.array_equal(s.view(np.uint32), s17[:, :k].view(np.uint32)), (rows, k)
                    assert np.array_equal(r, r17[:, :k]), (rows, k)
                    _, s64, rr, cc = orc.search(X, Qp, k, base)
                    bad = orc.check_topk(s, r, c, s64, rr, cc, orc.rescore(X, Qp, r, c, base), 1e-5)
                    assert not bad, (rows, k, bad[:3])
            eng.drop_collection(name)


_SMALL_COMPLETION = r"""
import json, sys
import torch                      # first: the library then binds torch's HIP runtime
import numpy as np
sys.path.insert(0, ROOT)
import __graft_entry__ as ge
pkg = ge.load_package()
rng = np.random.default_rng(11)
V = rng.standard_normal((221, 768)).astype(np.float32)
Q = rng.standard_normal((40, 768)).astype(np.float32)
out = []
with pkg.VectorEngine(device=0) as eng:
    eng.create_collection("c1", 768, 0, 0)
    eng.upsert("c1", list(range(221)), V)
    for i in range(40):
        s, r, c = eng.search("c1", Q[i:i + 1], 5)
        out.append([s.view(np.uint32).tolist(), r.tolist(), c.tolist()])
print(json.dumps(out))
"""


@pytest.mark.parametrize("env", [{"VS_SPIN_US": "0"}, {"VS_DIRECT_COMPLETION": "0"},
                                 {"VS_QUERY_ARGS": "0"}])
def test_small_completion_word_fallbacks(pkg, env):
    """The one-launch small path publishes its keys through a completion word in
    mapped host memory (HostDirect). Forty calls on one staging slot (the word's
    sequence advancing) must give the same bits as with the word read only after
    the stream's event (VS_SPIN_US=0: no spin, event then word check), as the
    D2H copy path (VS_DIRECT_COMPLETION=0) and as the query copied to the
    device instead of sent in the kernel arguments (VS_QUERY_ARGS=0)."""
    import os
    base = _run_py(_SMALL_COMPLETION)
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        other = _run_py(_SMALL_COMPLETION)
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert base == other


def test_small_completion_concurrent(pkg, orc):
    """Threads searching small collections at once: each call on its own staging
    slot and completion word (contexts and slots shared); every reply equals
    the serial one, bit for bit."""
    import threading
    rng = np.random.default_rng(5)
    with pkg.VectorEngine(device=0) as eng:
        names = []
        for i, rows in enumerate((221, 64, 200)):
            n = f"cc{i}"
            eng.create_collection(n, 768, 0, i % 2)
            eng.upsert(n, list(range(rows)), rng.standard_normal((rows, 768)).astype(np.float32))
            names.append(n)
        Q = rng.standard_normal((96, 768)).astype(np.float32)
        jobs = [(names[i % 3], i, 1 + i % 16) for i in range(96)]
        want = {j: eng.search(n, Q[j:j + 1], k) for n, j, k in jobs}
        got, errs = {}, []

        def worker(part):
            try:
                for _ in range(5):
                    for n, j, k in part:
                        got[j] = eng.search(n, Q[j:j + 1], k)
                        w = want[j]
                        if not (np.array_equal(got[j][0].view(np.uint32), w[0].view(np.uint32))
                                and np.array_equal(got[j][1], w[1])):
                            errs.append((n, j, k))
            except Exception as e:  # noqa: BLE001
                errs.append(repr(e))

        th = [threading.Thread(target=worker, args=(jobs[t::8],)) for t in range(8)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs[:5]


_GEMV_ONE = r"""
import json, sys
import torch                      # first: the library then binds torch's HIP runtime
import numpy as np
sys.path.insert(0, ROOT)
import __graft_entry__ as ge
pkg = ge.load_package()
out = {}
with pkg.VectorEngine(device=0) as eng:
    for dim, dtype, metric, rows in ((768, 0, 0, 300), (768, 1, 1, 5000), (1024, 1, 0, 70000),
                                     (128, 0, 1, 20000), (1536, 0, 0, 4000), (768, 0, 0, 200000)):
        name = f"g{dim}_{dtype}_{metric}_{rows}"
        eng.create_collection(name, dim, metric, dtype, 0, 1000)
        eng.generate(name, rows, 77)
        rng = np.random.default_rng(dim + rows)
        Q = (rng.standard_normal((6, dim)) * 3).astype(np.float32)
        allow = rng.random(rows) < 0.6
        for k in (1, 10, 17, 64, 65, 100, 128):
            for i in range(Q.shape[0]):
                s, r, c = eng.search(name, Q[i:i + 1], k)
                out[f"{name}/{k}/{i}"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
            s, r, c = eng.search_filtered(name, Q[:1], k, allow)
            out[f"{name}/{k}/f"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
        eng.drop_collection(name)
print(json.dumps(out))
"""


def test_gemv_one_launch_equals_three_launches(pkg):
    """One query on the GEMV list path runs as ONE launch (every workgroup
    preprocesses the raw query, the last one merges the workgroup lists) and,
    through the host API, hands its keys over by the completion word. Its
    answers must be bit-identical to query prep + scan + merge (VS_GEMV_ONE=0)
    over dims 128..1024 (1536: the three launches in both runs), both dtypes and
    metrics, 300..200k rows, k 1..128
    (KPL 1 and 2), with a row_base and with a shipped filter bitmap."""
    import os
    base = _run_py(_GEMV_ONE)
    os.environ["VS_GEMV_ONE"] = "0"
    try:
        other = _run_py(_GEMV_ONE)
    finally:
        os.environ.pop("VS_GEMV_ONE", None)
    assert base.keys() == other.keys()
    bad = [key for key in base if base[key] != other[key]]
    assert not bad, bad[:5]


_QMAX = r"""
import json, sys
import torch                      # first: the library then binds torch's HIP runtime
import numpy as np
sys.path.insert(0, ROOT)
import __graft_entry__ as ge
pkg = ge.load_package()
out = {}
with pkg.VectorEngine(device=0) as eng:
    # candidate MFMA path shapes: 8+ tiles per workgroup (>= 65k rows), both
    # dtypes, D = 768 / 1024 / 128, k 1 .. 128, filters, a row_base, and
    # 200k identical rows (every quarter full: the replacement path)
    for dim, dtype, metric, rows, base in ((768, 1, 1, 1_000_000, 0), (768, 0, 0, 300_000, 0),
                                           (1024, 1, 0, 400_000, 7000), (128, 1, 1, 2_000_000, 0)):
        name = f"q{dim}_{dtype}_{rows}"
        eng.create_collection(name, dim, metric, dtype, rows, base)
        eng.generate(name, rows, 5)
        rng = np.random.default_rng(dim + rows)
        Q = rng.standard_normal((300, dim)).astype(np.float32)
        allow = rng.random(rows) < 0.3
        for nq, k in ((256, 10), (300, 1), (64, 50), (200, 100), (33, 128), (2, 10)):
            s, r, c = eng.search(name, Q[:nq], k)
            out[f"{name}/{nq}/{k}"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
        s, r, c = eng.search_filtered(name, Q[:128], 20, allow)
        out[f"{name}/f"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
        eng.drop_collection(name)
    eng.create_collection("same", 128, 0, 1, 200_000)
    v = np.random.default_rng(1).standard_normal((1, 128)).astype(np.float32)
    eng.upsert("same", np.arange(200_000), np.repeat(v, 200_000, axis=0))
    Q = np.concatenate([v, np.random.default_rng(2).standard_normal((40, 128)).astype(np.float32)])
    for k in (10, 64, 128):
        s, r, c = eng.search("same", Q, k)
        out[f"same/{k}"] = [s.view(np.uint32).tolist(), r.tolist(), c.tolist()]
print(json.dumps(out))
"""


def test_select_quarter_maxima_equals_full_select(pkg):
    """r04: the main pass records every candidate quarter's largest score and
    the slab select reads only the quarters that can hold a top-k key. Its
    answers must be bit-identical to the select that re-reads every slab
    (VS_SELECT_QMAX=0): both dtypes, D 128 / 768 / 1024, k 1 .. 128, filters,
    a row_base, and full quarters (200k identical rows)."""
    import os
    base = _run_py(_QMAX)
    for var, val in (("VS_SELECT_QMAX", "0"),):
        os.environ[var] = val
        try:
            other = _run_py(_QMAX)
        finally:
            os.environ.pop(var, None)
        assert base.keys() == other.keys()
        bad = [key for key in base if base[key] != other[key]]
        assert not bad, (var, bad[:5])
