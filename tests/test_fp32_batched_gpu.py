"""Batched search of fp32 collections on v_mfma_f32_16x16x4_f32.

fp32 is the reference's collection type (rag/vector-service/main.go:102-112
creates collections with no datatype, i.e. Qdrant's default f32) and config
C2's dtype. A batch of >= 4 queries streams each corpus tile once for up to
128 queries (D <= 768; 256 at D <= 384) with exact f32 products and fp32
accumulation, then the same sample bound, candidate buffers and select as
the bf16 path. Checked against the exact fp64 oracle at the north_star fp32
tolerance (1e-5 relative).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _check(orc, s, r, c, s64, rr, cc, resc):
    bad = orc.check_topk(s, r, c, s64, rr, cc, resc, score_rtol=1e-5)
    assert not bad, bad[:8]


@pytest.mark.timeout(600)
def test_fp32_batched_1m_256_queries(engine, orc, pkg):
    n, dim, B = 1_000_000, 768, 256
    name = "f32_1m"
    engine.create_collection(name, dim, pkg.METRIC_COSINE, pkg.DTYPE_F32, n)
    try:
        engine.generate(name, n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 0, B, dim) * 0.5  # cosine normalises them back
        Qp = orc.preprocess(Q, cosine=True, bf16=False)
        for k in (10, 100):
            s, r, c = engine.search(name, Q, k)
            s64, rr, cc = orc.search_generated(orc.SEED_CORPUS, 0, n, Qp, k, False)
            resc = orc.rescore_generated(orc.SEED_CORPUS, Qp, r, c, False)
            _check(orc, s, r, c, s64, rr, cc, resc)
    finally:
        engine.drop_collection(name)


@pytest.mark.parametrize("dim", [128, 256, 384, 512, 768])
@pytest.mark.parametrize("nq,k", [(4, 10), (77, 1), (128, 16), (129, 50), (300, 128)])
def test_fp32_batched_dims(engine, orc, dim, nq, k):
    n = 150_000 if dim <= 384 else 60_000
    name = f"f32b_{dim}"
    engine.create_collection(name, dim, 0, 0, n)
    try:
        engine.generate(name, n, orc.SEED_CORPUS)
        Q = orc.generate(orc.SEED_QUERY, 31, nq, dim)
        s, r, c = engine.search(name, Q, k)
        X = orc.generate(orc.SEED_CORPUS, 0, n, dim)
        Qp = orc.preprocess(Q, True, False)
        s32, s64, rr, cc = orc.search(X, Qp, k)
        _check(orc, s, r, c, s64, rr, cc, orc.rescore(X, Qp, r, c))
    finally:
        engine.drop_collection(name)


def test_fp32_batched_small_collection_and_ties(engine, orc):
    """Small collections take the sorted-list pass (k <= 16) or per-query
    GEMV; exact duplicates must come back in row order; 40k identical rows
    fill the candidate quarters (in-place replacement)."""
    dim = 768
    base = orc.generate(orc.SEED_CORPUS, 0, 3000, dim)
    engine.create_collection("f32s", dim, 0, 0)
    engine.upsert("f32s", np.arange(3000), base)
    Q = orc.generate(orc.SEED_QUERY, 3, 9, dim)
    for k in (5, 16, 40):
        s, r, c = engine.search("f32s", Q, k)
        X = orc.preprocess(base, True, False)
        Qp = orc.preprocess(Q, True, False)
        s32, s64, rr, cc = orc.search(X, Qp, k)
        _check(orc, s, r, c, s64, rr, cc, orc.rescore(X, Qp, r, c))
    engine.drop_collection("f32s")
    n = 40_000
    same = np.tile(base[7:8], (n, 1))
    engine.create_collection("f32t", dim, 0, 0, n)
    engine.upsert("f32t", np.arange(n), same)
    Q = np.concatenate([base[7:8], orc.generate(orc.SEED_QUERY, 11, 7, dim)])
    for k in (10, 16, 50):
        s, r, c = engine.search("f32t", Q, k)
        assert np.all(r == np.arange(k)[None, :]), k  # ties: row ascending
        assert np.all(c == k)
    engine.drop_collection("f32t")


def test_fp32_batched_filtered(engine, orc, pkg):
    """The filter pre-mask on the fp32 MFMA passes (dense masks stream every
    row; masked rows are never candidates)."""
    n, dim = 200_000, 512
    engine.create_collection("f32f", dim, 0, 0, n)
    engine.generate("f32f", n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim)
    rng = np.random.default_rng(8)
    Q = orc.generate(orc.SEED_QUERY, 90, 64, dim)
    Qp = orc.preprocess(Q, True, False)
    for dens in (0.5, 0.2):
        mask = rng.random(n) < dens
        s, r, c = engine.search_filtered("f32f", Q, 10, mask)
        idx = np.flatnonzero(mask)
        s32, s64, rr, cc = orc.search(X[idx], Qp, 10)
        rr = idx[rr.astype(np.int64)].astype(np.uint64)
        loc = np.searchsorted(idx, r.astype(np.int64))
        resc = orc.rescore(X[idx], Qp, loc.astype(np.uint64), c)
        assert np.all(mask[r.astype(np.int64)])
        _check(orc, s, r, c, s64, rr, cc, resc)
    engine.drop_collection("f32f")
