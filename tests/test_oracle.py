"""The oracle itself: analytic known-answer tests, C vs numpy agreement, and the
committed golden fixtures (CPU only).

The reference has no tests or fixtures for this path, so
the oracle is pinned by (1) closed-form cosine/dot answers that follow from the
reference's collection config (Distance_Cosine, rag/vector-service/main.go:108)
and Qdrant's documented preprocess, and (2) two independent restatements (C
and numpy) agreeing bit for bit.
"""
import hashlib
import json
import os

import numpy as np
import pytest

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _digest(a):
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


# ---------------------------------------------------------------- generator
def test_generator_c_matches_numpy(orc):
    for bf16 in (False, True):
        a = orc.generate(orc.SEED_CORPUS, 12345, 64, 768, bf16=bf16)
        b = orc.np_generate(orc.SEED_CORPUS, 12345, 64, 768, bf16=bf16)
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_generator_rows_are_unit(orc):
    x = orc.generate(orc.SEED_CORPUS, 0, 256, 1024).astype(np.float64)
    assert np.allclose((x * x).sum(1), 1.0, atol=1e-6)


def test_generator_digest_pinned(orc):
    d = json.load(open(os.path.join(GOLDEN, "digests.json")))
    assert _digest(orc.generate(orc.SEED_CORPUS, 0, 4096, 768)) == d["corpus_f32_sha256"]
    assert _digest(orc.generate_raw(orc.SEED_CORPUS, 0, 4096, 768, True)) == d["corpus_bf16_sha256"]
    assert _digest(orc.generate(orc.SEED_QUERY, 0, 32, 768)) == d["queries_f32_sha256"]


def test_generator_head_fixture(orc):
    g = np.load(os.path.join(GOLDEN, "gen_head.npz"))
    assert np.array_equal(orc.generate(orc.SEED_CORPUS, 0, 8, 768), g["corpus_f32"])
    assert np.array_equal(orc.generate_raw(orc.SEED_CORPUS, 0, 8, 768, True), g["corpus_bf16_bits"])
    assert np.array_equal(orc.np_gen_ints(orc.SEED_CORPUS, 0, 1, 768)[0], g["ints_row0"])


def test_generator_shards_compose(orc):
    # row-sharded generation (global row numbers) == unsharded generation
    full = orc.generate(orc.SEED_CORPUS, 0, 100, 128)
    parts = [orc.generate(orc.SEED_CORPUS, lo, hi - lo, 128) for lo, hi in ((0, 37), (37, 100))]
    assert np.array_equal(full, np.concatenate(parts))


# --------------------------------------------------------------- bf16 / keys
def test_bf16_rne(orc):
    vals = np.array([1.0, 1.00390625, 1.0078125, 1.01171875, -3.14159, 1e-40, 65504.0,
                     np.inf, -np.inf], np.float32)
    got = orc.np_bf16_round(vals)
    for v, g in zip(vals, got):
        b = orc.lib().oracle_f32_to_bf16(float(v))
        assert np.uint32(b) << 16 == g.view(np.uint32)
    # ties to even: 1 + 2^-8 is halfway between 1 and 1 + 2^-7 -> 1
    assert got[1] == 1.0
    assert got[3] == np.float32(1.015625)
    assert np.isnan(orc.np_bf16_round(np.array([np.nan], np.float32)))[0]


# ---------------------------------------------------------------- preprocess
def test_preprocess_c_matches_numpy(orc):
    rng = np.random.default_rng(0)
    x = rng.standard_normal((50, 770)).astype(np.float32) * rng.uniform(1e-3, 1e3, (50, 1)).astype(np.float32)
    for cosine in (True, False):
        for bf16 in (False, True):
            a = orc.preprocess(x, cosine, bf16)
            b = orc.np_preprocess(x, cosine, bf16)
            assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


def test_preprocess_edge_fixture(orc):
    g = np.load(os.path.join(GOLDEN, "preprocess_edge.npz"))
    raw = g["raw"]
    assert np.array_equal(orc.preprocess(raw, True, False), g["cosine_f32"])
    assert np.array_equal(orc.preprocess(raw, True, True), g["cosine_bf16"])
    assert np.array_equal(orc.preprocess(raw, False, False), g["dot_f32"])
    out = g["cosine_f32"]
    assert np.all(out[0] == 0)                              # zero vector kept
    assert np.array_equal(out[1], raw[1])                   # |x|^2 < FLT_EPSILON kept
    assert np.array_equal(out[2], raw[2])                   # already unit: kept
    for i in (3, 4, 5):
        assert abs(float((out[i].astype(np.float64) ** 2).sum()) - 1) < 1e-6
    assert np.array_equal(g["dot_f32"], raw)                # Dot: no preprocessing


# ------------------------------------------------------- known-answer search
def _search(orc, X, q, k, cosine=True):
    Xp = orc.preprocess(np.asarray(X, np.float32), cosine)
    Qp = orc.preprocess(np.atleast_2d(np.asarray(q, np.float32)), cosine)
    return orc.search(Xp, Qp, k)


def test_kat_cosine_3d(orc):
    # stored [e0, e1, e2, e0+e1, -e0], query e0 (cf. README.md:725-738's 3-d probe)
    X = [[1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 1, 0], [-1, 0, 0]]
    s32, s64, rows, cnt = _search(orc, X, [1, 0, 0], 5)
    assert cnt[0] == 5
    assert rows[0].tolist() == [0, 3, 1, 2, 4]              # 0-score tie: row ascending
    assert np.allclose(s64[0], [1.0, 2 ** -0.5, 0.0, 0.0, -1.0], atol=1e-7)


def test_kat_cosine_scale_invariant(orc):
    rng = np.random.default_rng(3)
    X = rng.standard_normal((200, 96)).astype(np.float32)
    q = rng.standard_normal(96).astype(np.float32)
    a = _search(orc, X, q, 10)
    b = _search(orc, X * 7.0, q * 0.25, 10)
    assert np.array_equal(a[2], b[2])
    assert np.allclose(a[1], b[1], rtol=1e-6)


def test_kat_self_match(orc):
    X = orc.generate(orc.SEED_CORPUS, 0, 500, 768)
    s32, s64, rows, cnt = orc.search(X, X[[17, 250]], 3)
    assert rows[:, 0].tolist() == [17, 250]
    assert np.allclose(s64[:, 0], 1.0, atol=1e-6)


def test_kat_dot_is_plain_inner_product(orc):
    X = np.array([[1, 2, 3], [4, 5, 6], [-1, 0, 1]], np.float32)
    s32, s64, rows, cnt = _search(orc, X, [2, 0, 0], 3, cosine=False)
    assert rows[0].tolist() == [1, 0, 2]
    assert s64[0].tolist() == [8.0, 2.0, -2.0]


def test_kat_k_larger_than_rows_and_empty(orc):
    X = np.eye(4, 8, dtype=np.float32)
    s32, s64, rows, cnt = _search(orc, X, np.ones(8), 10)
    assert cnt[0] == 4 and rows[0, :4].tolist() == [0, 1, 2, 3]
    s32, s64, rows, cnt = orc.search(np.zeros((0, 8), np.float32), np.ones((1, 8), np.float32), 5)
    assert cnt[0] == 0


def test_kat_duplicates_tie_by_row(orc):
    base = orc.generate(orc.SEED_CORPUS, 0, 10, 64)
    X = np.concatenate([base, base[[3, 3, 3]]])             # rows 10,11,12 duplicate row 3
    s32, s64, rows, cnt = orc.search(X, base[[3]], 4)
    assert rows[0].tolist() == [3, 10, 11, 12]


def test_kat_zero_query(orc):
    X = orc.generate(orc.SEED_CORPUS, 0, 20, 32)
    s32, s64, rows, cnt = _search(orc, X, np.zeros(32), 5)
    assert rows[0].tolist() == [0, 1, 2, 3, 4] and np.all(s64 == 0)


# ------------------------------------------------------------ C vs numpy
@pytest.mark.parametrize("bf16", [False, True])
def test_search_c_matches_numpy(orc, bf16):
    X = orc.generate(orc.SEED_CORPUS, 0, 3000, 256, bf16=bf16)
    Q = orc.preprocess(orc.generate(orc.SEED_QUERY, 0, 8, 256), True, bf16)
    s32, s64, rows, cnt = orc.search(X, Q, 25)
    ns, nr = orc.np_search(X, Q, 25)
    assert np.array_equal(rows, nr)
    assert np.allclose(s64, ns, rtol=1e-12, atol=1e-15)


def test_golden_search(orc):
    g = np.load(os.path.join(GOLDEN, "search_4096x768.npz"))
    Q = orc.generate(orc.SEED_QUERY, 0, 32, 768)
    for tag, bf16 in (("f32", False), ("bf16", True)):
        X = orc.generate(orc.SEED_CORPUS, 0, 4096, 768, bf16=bf16)
        Qp = orc.preprocess(Q, True, bf16)
        assert np.array_equal(Qp, g[f"qpre_{tag}"])
        for k in (1, 5, 10, 100):
            s32, s64, rows, cnt = orc.search(X, Qp, k)
            assert np.array_equal(rows, g[f"rows_{tag}_k{k}"])
            assert np.array_equal(s64, g[f"scores64_{tag}_k{k}"])


def test_cpu_baseline_scan_agrees(orc):
    # the timed CPU baseline (fp32 multi-accumulator scan) ranks like the oracle
    Xraw = orc.generate_raw(orc.SEED_CORPUS, 0, 5000, 768, True)
    X = orc.generate(orc.SEED_CORPUS, 0, 5000, 768, True)
    Q = orc.preprocess(orc.generate(orc.SEED_QUERY, 0, 4, 768), True, True)
    s, r, nth = orc.cpu_scan(Xraw, True, Q, 10, threads=2)
    s32, s64, rows, cnt = orc.search(X, Q, 10)
    resc = orc.rescore(X, Q, r, np.full(4, 10, np.uint32))
    assert nth == 2
    assert not orc.check_topk(s, r, np.full(4, 10), s64, rows, cnt, resc, score_rtol=1e-5)


def test_check_topk_detects_errors(orc):
    X = orc.generate(orc.SEED_CORPUS, 0, 1000, 64)
    Q = orc.generate(orc.SEED_QUERY, 0, 2, 64)
    s32, s64, rows, cnt = orc.search(X, Q, 5)
    ok = orc.check_topk(s32, rows, cnt, s64, rows, cnt, s64, 1e-5)
    assert ok == []
    bad_rows = rows.copy()
    bad_rows[0, 0], bad_rows[0, 4] = rows[0, 4], rows[0, 0]
    resc = orc.rescore(X, Q, bad_rows, cnt)
    assert orc.check_topk(s32, bad_rows, cnt, s64, rows, cnt, resc, 1e-5)
    bad_s = s32.copy()
    bad_s[1, 2] *= 1.001
    assert orc.check_topk(bad_s, rows, cnt, s64, rows, cnt, s64, 1e-5)


def test_checksum_c_matches_numpy(orc):
    rng = np.random.default_rng(5)
    for n in (0, 1, 7, 8, 9, 15, 16, 17, 1000, 4099, 65536 + 3):
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert orc.checksum(d) == orc.np_checksum(d), n


def test_checksum_known_answers(orc):
    """Pinned by splitmix64's published outputs: one word w at index 0 hashes
    to splitmix64(w); splitmix64(1) = 0x910A2DEC89025CC1 (seed-1 first output
    of Vigna's reference splitmix64.c), splitmix64(0) = 0xE220A8397B1DCDAF."""
    assert orc.checksum(b"") == 0
    assert orc.checksum(b"\x01") == 0x910A2DEC89025CC1
    assert orc.checksum(b"\x00" * 8) == 0xE220A8397B1DCDAF
    # zero padding of the last word, position dependence, order-free sum
    assert orc.checksum(b"\x01\x00\x00") == orc.checksum(b"\x01")
    a, b = b"\x05" * 8, b"\x09" * 8
    assert orc.checksum(a + b) != orc.checksum(b + a)
    assert orc.checksum(a + b) == (orc.checksum(a) + orc.checksum(b"\0" * 8 + b)
                                   - orc.checksum(b"\0" * 8)) % 2 ** 64
