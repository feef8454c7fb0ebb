"""Seeded random shapes against the oracle (r04): every search path of the
engine (small one-launch scan, one-query GEMV chain, lists / candidate MFMA
passes with their selects, large-k score pass + radix select, gathered
filters) is reached by some case, in combinations the hand-picked tests do
not name. Each case draws dim, dtype, metric, rows, row_base, queries, k and
a filter from a fixed seed, so a failure names a reproducible case.

Bar (BASELINE.json north_star, oracle.check_topk): rows equal the oracle's
except exact-score near-ties < 1e-5 relative; scores within 1e-5 relative of
the exact fp64 score. Anchor: Points.Search, rag/vector-service/main.go:249-254.
"""
import numpy as np
import pytest

DIMS = (100, 128, 256, 384, 512, 768, 1024, 1536)
ROWS = (1, 17, 300, 4_000, 70_000, 260_000)
NQ = (1, 2, 5, 64, 256, 300)
KS = (1, 5, 10, 16, 17, 50, 100, 128, 129, 600)


def _case(i):
    rng = np.random.default_rng(1000 + i)
    dim = int(rng.choice(DIMS))
    rows = int(rng.choice(ROWS))
    while rows * dim > 200_000_000:  # host copy for the oracle: <= 0.8 GB fp32
        rows = int(rng.choice(ROWS))
    nq = int(rng.choice(NQ))
    k = int(rng.choice(KS))
    if k > 128 and nq * rows * dim > 3e9:  # the large-k path runs one pass per query
        nq = 2
    return {"dim": dim, "rows": rows, "nq": nq, "k": k, "dtype": int(rng.integers(0, 2)),
            "metric": int(rng.integers(0, 2)), "row_base": int(rng.choice([0, 0, 12345])),
            "filter": str(rng.choice(["none", "none", "dense", "sparse"])),
            "seed": int(rng.integers(1, 1 << 30))}


@pytest.mark.gpu
@pytest.mark.parametrize("i", range(36))
def test_fuzz_case(engine, orc, i):
    c = _case(i)
    name = f"fz{i}"
    dim, rows, nq, k = c["dim"], c["rows"], c["nq"], c["k"]
    bf16, cosine = bool(c["dtype"]), c["metric"] == 0
    base = c["row_base"]
    engine.create_collection(name, dim, c["metric"], c["dtype"], rows, base)
    try:
        engine.generate(name, rows, c["seed"])  # global rows base .. base + rows - 1
        X = orc.generate(c["seed"], base, rows, dim, bf16=bf16)
        rng = np.random.default_rng(c["seed"])
        Q = (rng.standard_normal((nq, dim)) * rng.uniform(0.5, 3.0)).astype(np.float32)
        Qp = orc.preprocess(Q, cosine, bf16)
        if c["filter"] == "none":
            s, r, cnt = engine.search(name, Q, k)
            _, s64, rr, cc = orc.search(X, Qp, k, base)
            resc = orc.rescore(X, Qp, r, cnt, base)
        else:
            mask = rng.random(rows) < (0.5 if c["filter"] == "dense" else 0.02)
            s, r, cnt = engine.search_filtered(name, Q, k, mask)
            idx = np.flatnonzero(mask)  # ascending: subset order = row order
            _, s64, rl, cc = orc.search(X[idx], Qp, k)
            valid = np.arange(k)[None, :] < cc[:, None]
            rr = np.zeros_like(rl)
            if len(idx):
                rr = np.where(valid, idx[np.where(valid, rl, 0).astype(np.int64)] + base,
                              0).astype(np.uint64)
            loc = r.astype(np.int64) - base
            dvalid = np.arange(k)[None, :] < cnt[:, None]
            assert np.all(mask[loc[dvalid]]), c  # every returned row is allowed
            pos = np.searchsorted(idx, np.where(dvalid, loc, 0)).astype(np.uint64)
            resc = orc.rescore(X[idx], Qp, pos, cnt)
        bad = orc.check_topk(s, r, cnt, s64, rr, cc, resc, score_rtol=1e-5)
        assert not bad, (c, bad[:6])
    finally:
        engine.drop_collection(name)


def test_fuzz_covers_every_path():
    """(CPU) The 36 drawn cases reach every path: one query and batches, k on both
    sides of 16 / 128, small and MFMA-sized collections, filters, row_base,
    bf16 and fp32, both metrics (the draw is deterministic; this pins it)."""
    cs = [_case(i) for i in range(36)]
    assert any(c["nq"] == 1 for c in cs) and any(c["nq"] >= 64 for c in cs)
    assert any(c["k"] > 128 for c in cs) and any(c["k"] <= 16 for c in cs)
    assert any(17 <= c["k"] <= 128 for c in cs)
    assert any(c["rows"] >= 70_000 and c["nq"] >= 2 for c in cs)
    assert any(c["rows"] <= 300 for c in cs)
    assert {c["filter"] for c in cs} == {"none", "dense", "sparse"}
    assert {c["dtype"] for c in cs} == {0, 1} and {c["metric"] for c in cs} == {0, 1}
    assert any(c["row_base"] for c in cs)
