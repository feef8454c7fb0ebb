"""Payload filter pre-mask through vs_search_filtered.

The bitmap is applied inside every scan kernel (GEMV, MFMA sample / candidate
/ sorted-list passes and the full-quarter replacement); the result must be the
oracle's exact top k over the allowed rows only, with the same (score desc,
row asc) order.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCORE_RTOL = 1e-5


def _masked_parity(orc, X, Qp, s, r, c, k, mask):
    idx = np.flatnonzero(mask)
    s32, s64, rows, cnt = orc.search(np.ascontiguousarray(X[idx]), Qp, k)
    rows = idx[rows.astype(np.int64)].astype(np.uint64)
    rows[np.arange(k)[None, :] >= cnt[:, None]] = 0
    assert np.all(mask[r[c[:, None] > np.arange(k)[None, :]].astype(np.int64)]), "masked row returned"
    resc = orc.rescore(X, Qp, r, c)
    bad = orc.check_topk(s, r, c, s64, rows, cnt, resc, SCORE_RTOL)
    assert not bad, bad[:10]


@pytest.fixture(scope="module")
def fcorpus(engine, orc):
    n, dim = 200_000, 768
    engine.create_collection("filt", dim, 0, 1, n)
    engine.generate("filt", n, orc.SEED_CORPUS)
    yield "filt", orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=True)
    engine.drop_collection("filt")


@pytest.mark.parametrize("density", [0.5, 0.05, 0.002])
@pytest.mark.parametrize("nq,k", [(1, 10), (256, 10), (300, 16), (64, 100)])
def test_filtered_search_bf16(engine, orc, fcorpus, density, nq, k):
    """nq = 1: GEMV; nq >= 2: sample + candidate MFMA passes (k > 16 and a
    selective mask may fill candidate quarters: in-place replacement)."""
    name, X = fcorpus
    rng = np.random.default_rng(int(density * 1e4) + nq + k)
    mask = rng.random(X.shape[0]) < density
    Q = orc.generate(orc.SEED_QUERY, 2000 + nq, nq, 768)
    s, r, c = engine.search_filtered(name, Q, k, mask)
    assert np.all(c == min(k, int(mask.sum())))
    _masked_parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k, mask)


def test_filter_blocks_and_edges(engine, orc, fcorpus, pkg):
    name, X = fcorpus
    n = X.shape[0]
    Q = orc.generate(orc.SEED_QUERY, 9, 40, 768)
    # a contiguous block (whole tiles / workgroups masked) plus single rows
    mask = np.zeros(n, bool)
    mask[70_000:90_000] = True
    mask[[0, 31, 32, 63, 64, n - 1]] = True
    s, r, c = engine.search_filtered(name, Q, 10, mask)
    _masked_parity(orc, X, orc.preprocess(Q, True, True), s, r, c, 10, mask)
    # all rows allowed == the unfiltered search, bit for bit
    a = engine.search(name, Q, 10)
    b = engine.search_filtered(name, Q, 10, np.ones(n, bool))
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    # nothing allowed: no results
    for nq in (1, 40):
        s, r, c = engine.search_filtered(name, Q[:nq], 10, np.zeros(n, bool))
        assert np.all(c == 0)
    # fewer allowed rows than k
    few = np.zeros(n, bool)
    few[[5, 150_000, 199_999]] = True
    s, r, c = engine.search_filtered(name, Q, 10, few)
    assert np.all(c == 3) and set(r[0, :3].tolist()) == {5, 150_000, 199_999}
    with pytest.raises(pkg.VSError):
        engine.search_filtered(name, Q, 10, pkg.pack_allow(np.ones(n - 64, bool)))  # too short


@pytest.mark.parametrize("dtype,nq", [(0, 1), (0, 7), (1, 33)])
def test_filtered_small_collections(engine, orc, dtype, nq):
    """fp32 (GEMV per query) and a small bf16 collection (sorted-list MFMA pass)."""
    n, dim = 20_000, 768
    name = f"fsmall_{dtype}"
    engine.create_collection(name, dim, 0, dtype)
    engine.generate(name, n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, dim, bf16=bool(dtype))
    mask = np.random.default_rng(3).random(n) < 0.1
    Q = orc.generate(orc.SEED_QUERY, 77, nq, dim)
    s, r, c = engine.search_filtered(name, Q, 10, mask)
    _masked_parity(orc, X, orc.preprocess(Q, True, bool(dtype)), s, r, c, 10, mask)
    engine.drop_collection(name)


def test_filtered_full_quarters(engine, orc):
    """Ties under a mask: the allowed identical rows fill the candidate
    buffers' quarters; the in-place replacement compares masked slab maxima,
    so filtered-out rows never displace allowed ones."""
    n, dim = 70_000, 768
    base = orc.generate(orc.SEED_CORPUS, 0, n, dim)
    base[:40_000] = base[12_345]
    engine.create_collection("fties", dim, 0, 1, n)
    engine.upsert("fties", np.arange(n), base)
    X = orc.preprocess(base, True, True)
    mask = np.ones(n, bool)
    mask[:20_000:2] = False  # half of the first tied rows are filtered out
    Q = np.concatenate([base[12_345:12_346], orc.generate(orc.SEED_QUERY, 7, 20, dim)])
    for k in (10, 50, 128):
        s, r, c = engine.search_filtered("fties", Q, k, mask)
        assert r[0].tolist() == [2 * i + 1 for i in range(k)]
        _masked_parity(orc, X, orc.preprocess(Q, True, True), s, r, c, k, mask)
    engine.drop_collection("fties")


@pytest.mark.parametrize("dtype,dim", [(0, 768), (1, 768), (0, 100), (1, 1024)])
def test_filtered_gather_path(engine, orc, pkg, dtype, dim):
    """Selective filters (<= 1/8 of the rows allowed) on the GEMV path scan a
    compacted row list instead of the whole collection (compact_rows_kernel +
    the GATHER scans): results must equal the oracle over the allowed rows,
    including exact ties (duplicated rows), every list width (k = 1, 100,
    1000 > allowed), the generic-dimension kernel (dim 100) and a mask whose
    last word is partial."""
    n = 48_037
    name = f"fgather_{dtype}_{dim}"
    base = orc.generate(orc.SEED_CORPUS, 0, n, dim)
    base[100:400] = base[7]  # 301 identical rows
    engine.create_collection(name, dim, 0, dtype, n)
    engine.upsert(name, np.arange(n), base)
    X = orc.preprocess(base, True, bool(dtype))
    rng = np.random.default_rng(dim + dtype)
    mask = rng.random(n) < 0.02
    mask[100:400:3] = True  # a third of the tied rows
    mask[[7, n - 1]] = True
    assert mask.sum() * 8 <= n
    Q = np.concatenate([base[7:8], orc.generate(orc.SEED_QUERY, 31, 2, dim)])
    Qp = orc.preprocess(Q, True, bool(dtype))
    for k in (1, 100, 1000):
        for nq in (1, 3):
            s, r, c = engine.search_filtered(name, Q[:nq], k, mask)
            assert np.all(c == min(k, int(mask.sum())))
            _masked_parity(orc, X, Qp[:nq], s, r, c, k, mask)
    # the tied rows come back in row order for the query equal to them
    s, r, c = engine.search_filtered(name, Q[:1], 50, mask)
    tied = [7] + [i for i in range(100, 400) if mask[i]]
    assert r[0, :50].tolist() == sorted(tied)[:50]
    # bits set past the last row (in the partial last word) must not leak rows
    words = pkg.pack_allow(mask)
    words[-1] |= ~np.uint64(0) << np.uint64(n % 64)
    s2, r2, c2 = engine.search_filtered(name, Q, 100, words)
    s1, r1, c1 = engine.search_filtered(name, Q, 100, mask)
    assert np.array_equal(r1, r2) and np.array_equal(c1, c2)
    engine.drop_collection(name)



def test_filtered_gather_batches(engine, orc):
    """A batch with a very selective filter on a large collection leaves the
    MFMA pass for per-query gathered scans (search_core: nq gathers cost less
    than one streamed pass). Only the allowed rows are generated on the host:
    a block, scattered single rows and the collection's last row."""
    n, dim = 2_000_000, 768
    engine.create_collection("fgbig", dim, 0, 1, n)
    engine.generate("fgbig", n, orc.SEED_CORPUS)
    rng = np.random.default_rng(5)
    idx = np.unique(np.concatenate([np.arange(700_000, 703_000),
                                    rng.choice(n, 1500, replace=False), [n - 1]]))
    mask = np.zeros(n, bool)
    mask[idx] = True
    Xa = np.concatenate([orc.generate(orc.SEED_CORPUS, 700_000, 3000, dim, bf16=True)] +
                        [orc.generate(orc.SEED_CORPUS, int(r), 1, dim, bf16=True)
                         for r in idx if not 700_000 <= r < 703_000])
    order = np.argsort(np.concatenate([np.arange(700_000, 703_000),
                                       [r for r in idx if not 700_000 <= r < 703_000]]))
    Xa = Xa[order]  # rows of idx, ascending
    for nq, k in ((8, 10), (4, 128), (2, 1)):
        Q = orc.generate(orc.SEED_QUERY, 600 + nq, nq, dim)
        Qp = orc.preprocess(Q, True, True)
        s, r, c = engine.search_filtered("fgbig", Q, k, mask)
        assert np.all(c == k)
        assert np.all(mask[r.astype(np.int64)]), "masked row returned"
        pos = np.searchsorted(idx, r.astype(np.int64)).astype(np.uint64)
        s32, s64, rows, cnt = orc.search(Xa, Qp, k)
        resc = orc.rescore(Xa, Qp, pos, c)
        bad = orc.check_topk(s, pos, c, s64, rows, cnt, resc, SCORE_RTOL)
        assert not bad, bad[:10]
    engine.drop_collection("fgbig")


def test_device_resident_filters(engine, orc, pkg, fcorpus):
    """vs_filter_create / vs_search_filter_id / vs_filter_drop: a filter kept
    in HBM (bitmap, and the compacted row list when selective) gives exactly
    what vs_search_filtered gives with the same bitmap, on the GEMV gather,
    GEMV streamed and MFMA paths; it is bound to the collection's row count
    and dies with vs_filter_drop."""
    name, X = fcorpus
    n = X.shape[0]
    rng = np.random.default_rng(21)
    Q = orc.generate(orc.SEED_QUERY, 808, 40, 768)
    ids = []
    for dens in (0.003, 0.1, 0.6, 0.0):
        mask = rng.random(n) < dens
        fid = engine.filter_create(name, mask)
        assert fid not in ids
        ids.append(fid)
        for nq, k in ((1, 10), (1, 200), (40, 10), (3, 100)):
            a = engine.search_filtered(name, Q[:nq], k, mask)
            b = engine.search_filter_id(name, Q[:nq], k, fid)
            assert all(np.array_equal(x, y) for x, y in zip(a, b)), (dens, nq, k)
    for fid in ids:
        engine.filter_drop(fid)
    with pytest.raises(pkg.VSError):
        engine.search_filter_id(name, Q[:1], 10, ids[0])  # dropped
    with pytest.raises(pkg.VSError):
        engine.filter_drop(ids[0])
    with pytest.raises(pkg.VSError):
        engine.filter_create(name, pkg.pack_allow(np.ones(n - 64, bool)))  # too short
    # bound to the row count at creation
    engine.create_collection("fres", 128, 0, 0)
    base = orc.generate(orc.SEED_CORPUS, 0, 5000, 128)
    engine.upsert("fres", np.arange(4000), base[:4000])
    fid = engine.filter_create("fres", np.arange(4000) % 7 == 0)
    s, r, c = engine.search_filter_id("fres", base[:2], 5, fid)
    assert np.all(r % 7 == 0) and r[0, 0] == 0
    with pytest.raises(pkg.VSError):
        engine.search_filter_id(name, Q[:1], 10, fid)  # another collection
    engine.upsert("fres", np.arange(4000, 5000), base[4000:])
    with pytest.raises(pkg.VSError):
        engine.search_filter_id("fres", base[:2], 5, fid)  # rows were added: stale
    engine.filter_drop(fid)
    # a filter dies with its collection: after a drop and a re-create with
    # the same name and row count its id is gone
    fid = engine.filter_create("fres", np.arange(5000) % 3 == 0)
    engine.drop_collection("fres")
    engine.create_collection("fres", 128, 0, 0)
    engine.upsert("fres", np.arange(5000), base)
    with pytest.raises(pkg.VSError) as ei:
        engine.search_filter_id("fres", base[:2], 5, fid)
    assert ei.value.code == -2  # not found: freed with the dropped collection
    engine.drop_collection("fres")
