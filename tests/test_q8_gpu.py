"""Int8 prefilter (r04; DESIGN.md §5 "int8 prefilter", vs_q8.hip): batched
searches of bf16 collections run an int8 MFMA pass that admits every row
whose proven upper bound reaches the sample bound, and the survivors are
rescored from the bf16 rows on the bf16 pass's own MFMA chain. The answer
must be the bf16 pass's, bit for bit:
checked here against the oracle after every kind of store-side write that
must keep the int8 copy in step (appends, shuffled overwrites with
duplicates, rows past the collection's int8 scale, the rescale at doubled
rows, snapshot / restore), and on the paths that hand a batch back to the
bf16 pass on the device (a zero query, quarters overflowing on equal rows).

Bar (BASELINE.json north_star, oracle.check_topk): rows equal the oracle's
except exact-score near-ties < 1e-5 relative; scores within 1e-5 relative.
Anchor: Points.Search, rag/vector-service/main.go:249-254.
"""
import numpy as np
import pytest

DIM = 768
SCORE_RTOL = 1e-5


def _parity(orc, X, Qp, s, r, c, k):
    _, s64, rows, cnt = orc.search(X, Qp, k)
    resc = orc.rescore(X, Qp, r, c)
    bad = orc.check_topk(s, r, c, s64, rows, cnt, resc, SCORE_RTOL)
    assert not bad, bad[:8]


@pytest.fixture(scope="module")
def pair(pkg):
    """Two engines over the same 300k x 768 bf16 rows (inner product):
    prefilter on (default) and off (VS_FLAG_NO_PREFILTER)."""
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    for e in (a, b):
        e.create_collection("p", DIM, pkg.METRIC_DOT, pkg.DTYPE_BF16, 300_000)
        e.generate("p", 300_000, 77)
    yield a, b
    a.close()
    b.close()


@pytest.mark.gpu
def test_prefilter_copy_is_kept(pair):
    a, b = pair
    assert a.prefilter_bytes("p") >= 300_000 * DIM
    assert b.prefilter_bytes("p") == 0


@pytest.mark.gpu
@pytest.mark.parametrize("nq,k", [(256, 10), (256, 100), (17, 1), (300, 128), (2, 50)])
def test_prefilter_equals_oracle_and_bf16_pass(pair, orc, nq, k):
    a, b = pair
    X = orc.generate(77, 0, 300_000, DIM, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 500, nq, DIM)
    Qp = orc.preprocess(Q, False, True)
    s1, r1, c1 = a.search("p", Q, k)
    _parity(orc, X, Qp, s1, r1, c1, k)
    s2, r2, c2 = b.search("p", Q, k)
    # survivors are rescored on the bf16 pass's own MFMA chain: bit for bit
    assert np.array_equal(c1, c2) and np.array_equal(r1, r2)
    assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("nq,k", [(256, 50), (100, 10), (3, 128)])
def test_prefilter_1024_cosine(pkg, orc, nq, k):
    """C5's row shape: 1024-d cosine rows, 128 queries per int8 launch."""
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        n = 160_000
        for e in (a, b):
            e.create_collection("c", 1024, pkg.METRIC_COSINE, pkg.DTYPE_BF16, n)
            e.generate("c", n, 55)
        assert a.prefilter_bytes("c") > 0 and b.prefilter_bytes("c") == 0
        X = orc.generate(55, 0, n, 1024, bf16=True)
        Q = orc.generate(orc.SEED_QUERY, 7000, nq, 1024)
        s1, r1, c1 = a.search("c", Q, k)
        _parity(orc, X, orc.preprocess(Q, True, True), s1, r1, c1, k)
        s2, r2, c2 = b.search("c", Q, k)
        assert np.array_equal(r1, r2) and np.array_equal(s1.view(np.uint32), s2.view(np.uint32))
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nq,k", [(256, 10), (300, 64), (129, 128), (5, 1)])
def test_prefilter_fp32_rows(pkg, orc, nq, k):
    """fp32 collections (the reference's own dtype): one int8 launch of up to
    256 queries over two 128-query f32 sample passes, survivors rescored on
    the f32 pass's 16x16x4 chain -- its keys, bit for bit."""
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        n = 150_000
        for e in (a, b):
            e.create_collection("f", DIM, pkg.METRIC_COSINE, pkg.DTYPE_F32, n)
            e.generate("f", n, 66)
        assert a.prefilter_bytes("f") > 0 and b.prefilter_bytes("f") == 0
        X = orc.generate(66, 0, n, DIM)
        Q = orc.generate(orc.SEED_QUERY, 8000, nq, DIM)
        s1, r1, c1 = a.search("f", Q, k)
        _parity(orc, X, orc.preprocess(Q, True, False), s1, r1, c1, k)
        s2, r2, c2 = b.search("f", Q, k)
        assert np.array_equal(r1, r2) and np.array_equal(s1.view(np.uint32), s2.view(np.uint32))
    finally:
        a.close()
        b.close()


@pytest.mark.gpu
@pytest.mark.parametrize("density,k", [(0.3, 10), (0.6, 100), (0.2, 1)])
def test_prefilter_filtered(pair, orc, density, k):
    """A pre-mask rides along the int8 pass (masked rows never a maximum or a
    survivor): the bf16 pass's filtered keys, bit for bit, and the oracle's."""
    a, b = pair
    rng = np.random.default_rng(int(density * 100) + k)
    n = 300_000
    mask = rng.random(n) < density
    X = orc.generate(77, 0, n, DIM, bf16=True)
    Q = orc.generate(orc.SEED_QUERY, 600, 256, DIM)
    s1, r1, c1 = a.search_filtered("p", Q, k, mask)
    s2, r2, c2 = b.search_filtered("p", Q, k, mask)
    assert np.array_equal(r1, r2) and np.array_equal(s1.view(np.uint32), s2.view(np.uint32))
    idx = np.flatnonzero(mask)
    Qp = orc.preprocess(Q, False, True)
    _, s64, rl, cc = orc.search(X[idx], Qp, k)
    valid = np.arange(k)[None, :] < cc[:, None]
    rr = np.where(valid, idx[np.where(valid, rl, 0).astype(np.int64)], 0).astype(np.uint64)
    assert np.all(mask[r1[np.arange(k)[None, :] < c1[:, None]].astype(np.int64)])
    pos = np.searchsorted(idx, r1.astype(np.int64)).astype(np.uint64)
    resc = orc.rescore(X[idx], Qp, pos, c1)
    bad = orc.check_topk(s1, r1, c1, s64, rr, cc, resc, SCORE_RTOL)
    assert not bad, bad[:8]


@pytest.mark.gpu
def test_prefilter_follows_every_write(pkg, orc, tmp_path):
    rng = np.random.default_rng(5)
    e = pkg.VectorEngine(device=0)
    try:
        n0 = 200_000
        e.create_collection("w", DIM, pkg.METRIC_DOT, pkg.DTYPE_BF16)
        e.generate("w", n0, 91)
        assert e.prefilter_bytes("w") > 0
        X = orc.generate(91, 0, n0, DIM, bf16=True)
        Q = (rng.standard_normal((8, DIM)) / np.sqrt(DIM)).astype(np.float32)
        Qp = orc.preprocess(Q, False, True)

        def check(k=10):
            s, r, c = e.search("w", Q, k)
            _parity(orc, X, Qp, s, r, c, k)
            return r

        check()
        # 1. shuffled overwrites with duplicates (the tile-list refresh): rows
        # made to match the queries must come out on top
        ids = rng.choice(n0, 3000, replace=True).astype(np.uint64)
        V = (0.2 * rng.standard_normal((len(ids), DIM)) / np.sqrt(DIM)).astype(np.float32)
        V[:8] += 3.0 * Q  # the first 8 overwritten rows align with the queries
        e.upsert("w", ids, V)
        u, first = np.unique(ids[::-1], return_index=True)
        X[u] = orc.preprocess(V[len(ids) - 1 - first], False, True)
        r = check()
        for i in range(8):
            if ids[i] not in ids[8:]:  # not overwritten again later in the call
                assert int(ids[i]) in set(r[i].tolist())
        # 2. an ascending append past the collection's int8 scale (clipped
        # values: measured error bounds) that holds the best rows
        big = (4.0 * rng.standard_normal((20_000, DIM)) / np.sqrt(DIM)).astype(np.float32)
        big[100:108] = 5.0 * Q
        e.upsert("w", np.arange(n0, n0 + len(big)), big)
        X = np.concatenate([X, orc.preprocess(big, False, True)])
        r = check(16)
        for i in range(8):
            assert n0 + 100 + i in set(r[i].tolist())
        # 3. rows doubled: the copy is rebuilt with a new scale
        e.generate("w", 250_000, 92)
        n1 = X.shape[0]
        X = np.concatenate([X, orc.generate(92, n1, 250_000, DIM, bf16=True)])
        check(50)
        # 4. snapshot / restore: the restored collection gets its own copy
        path = str(tmp_path / "w.snap")
        e.snapshot("w", path)
        e.restore("w2", path)
        assert e.prefilter_bytes("w2") > 0
        s, r, c = e.search("w2", Q, 10)
        _parity(orc, X, Qp, s, r, c, 10)
        e.drop_collection("w2")
    finally:
        e.close()


@pytest.mark.gpu
def test_prefilter_hands_batches_to_bf16_pass(pkg, orc):
    """A zero query (every dot 0: every row admitted) and 100k equal rows
    (quarters overflow) set the batch's gate; the bf16 pass behind it answers."""
    e = pkg.VectorEngine(device=0)
    try:
        n = 150_000
        e.create_collection("g", DIM, pkg.METRIC_DOT, pkg.DTYPE_BF16)
        X = orc.generate(31, 0, n, DIM, bf16=True)
        X[20_000:120_000] = X[5]
        e.upsert("g", np.arange(n), X)
        assert e.prefilter_bytes("g") > 0
        Q = orc.generate(orc.SEED_QUERY, 900, 6, DIM)
        Q[0] = 0.0
        Q[1] = X[5] * 2.0  # the equal rows lead
        Qp = orc.preprocess(Q, False, True)
        for k in (10, 64):
            s, r, c = e.search("g", Q, k)
            _parity(orc, X, Qp, s, r, c, k)
    finally:
        e.close()


def test_prefilter_flag_and_symbol(pkg):
    """(CPU) The flag and the accessor are part of the boundary."""
    assert pkg.FLAG_NO_PREFILTER == 32
    import re
    import os
    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "vsearch.h")).read()
    assert re.search(r"#define VS_FLAG_NO_PREFILTER 32u", hdr)
    assert "vs_collection_prefilter_bytes" in hdr


@pytest.mark.gpu
@pytest.mark.parametrize("k", [65, 100, 128])
def test_prefilter_large_k_ties(pkg, orc, k):
    """k > 64 (radix floors for the two rounds and the final sort): 700
    copies of one row that the queries favour make the k-th bucket all ties;
    the keys must still be the bf16 pass's (ties ordered by row)."""
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        n = 200_000
        X = orc.generate(41, 0, n, DIM, bf16=True)
        X[50_000:50_700] = X[7]
        for e in (a, b):
            e.create_collection("t", DIM, pkg.METRIC_DOT, pkg.DTYPE_BF16)
            e.upsert("t", np.arange(n), X)
        assert a.prefilter_bytes("t") > 0
        Q = orc.generate(orc.SEED_QUERY, 1200, 130, DIM)
        Q[::2] += 0.5 * X[7]
        s1, r1, c1 = a.search("t", Q, k)
        _parity(orc, X, orc.preprocess(Q, False, True), s1, r1, c1, k)
        s2, r2, c2 = b.search("t", Q, k)
        assert np.array_equal(r1, r2) and np.array_equal(s1.view(np.uint32), s2.view(np.uint32))
    finally:
        a.close()
        b.close()


_FAIL_SCRIPT = r"""
import sys
import numpy as np
sys.path.insert(0, sys.argv[1])
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
e = pkg.VectorEngine(device=0)
n0, dim = 200_000, 768
e.create_collection("f", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16)
e.generate("f", n0, 41)  # first copy: built (nothing to be stale yet)
assert e.prefilter_bytes("f") > 0
rng = np.random.default_rng(3)
Q = (rng.standard_normal((16, dim)) / np.sqrt(dim)).astype(np.float32)
ids = np.array([7, 150_001, 99_999], dtype=np.uint64)
V = np.stack([3.0 * Q[0], 3.0 * Q[1], 3.0 * Q[2]]).astype(np.float32)
failed = False
try:
    e.upsert("f", ids, V)  # the rows are written, the int8 refresh fails
except Exception as ex:
    failed = "injected" in str(ex)
assert failed, "the injected failure did not surface"
assert e.prefilter_bytes("f") == 0, "stale int8 copy kept after a failed refresh"
X = orc.generate(41, 0, n0, dim, bf16=True)
X[ids.astype(np.int64)] = orc.preprocess(V, False, True)
Qp = orc.preprocess(Q, False, True)
s, r, c = e.search("f", Q, 10)
_, s64, rows, cnt = orc.search(X, Qp, 10)
bad = orc.check_topk(s, r, c, s64, rows, cnt, orc.rescore(X, Qp, r, c), 1e-5)
assert not bad, bad[:4]
for i in range(3):
    assert int(ids[i]) == int(r[i, 0])
e.close()
print("ok")
"""


@pytest.mark.gpu
def test_prefilter_dropped_on_failed_refresh(tmp_path):
    """a failure after the store-side write (here injected with
    VS_Q8_FAIL_AFTER_WRITE=1, read once per process, so in a child process)
    must not leave a stale int8 copy whose bounds miss the new rows: the copy
    is dropped and batched searches answer from the bf16 pass."""
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "fail_refresh.py"
    script.write_text(_FAIL_SCRIPT)
    env = dict(os.environ, VS_Q8_FAIL_AFTER_WRITE="1")
    p = subprocess.run([sys.executable, str(script), root], env=env, capture_output=True,
                       text=True, timeout=240)
    assert p.returncode == 0 and p.stdout.strip().endswith("ok"), p.stdout[-2000:] + p.stderr[-2000:]


@pytest.mark.gpu
@pytest.mark.parametrize("copies,spread", [(3000, False), (20000, True), (500, True)])
def test_select_recomputes_lossy_quarters_and_streams_spills(pkg, orc, copies, spread):
    """r05: a quarter the int8 pass overflowed (its count past its capacity)
    is recomputed from the int8 copy by the select, and more survivors than
    the select's buffer stream through a running top k -- no gated bf16 pass
    behind the batch. Duplicated rows (RAG corpora repeat boilerplate chunks)
    force both: copies of one row, contiguous (one workgroup's quarters) or
    spread over the collection, with queries aligned to them and random ones.
    Keys equal the bf16 pass's bit for bit, and the oracle's."""
    n, dim = 300_000, DIM
    rng = np.random.default_rng(copies)
    X = orc.generate(61, 0, n, dim, bf16=True)
    dst = (rng.choice(n, copies, replace=False) if spread else np.arange(40_000, 40_000 + copies))
    X[dst] = X[11]
    a = pkg.VectorEngine(device=0)
    b = pkg.VectorEngine(device=0, prefilter=False)
    try:
        for e in (a, b):
            e.create_collection("o", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16)
            e.upsert("o", np.arange(n), X)
        assert a.prefilter_bytes("o") > 0
        Q = orc.generate(orc.SEED_QUERY, 3300, 40, dim)
        Q[:8] = X[11] * np.linspace(0.5, 2.0, 8)[:, None]  # the copies lead
        Q[8:12] = X[11] * 0.7 + Q[8:12] * 0.3
        Qp = orc.preprocess(Q, False, True)
        for k in (10, 64, 100):
            s1, r1, c1 = a.search("o", Q, k)
            s2, r2, c2 = b.search("o", Q, k)
            assert np.array_equal(c1, c2) and np.array_equal(r1, r2)
            assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32))
            _parity(orc, X, Qp, s1, r1, c1, k)
    finally:
        a.close()
        b.close()
