"""(CPU) The int8 prefilter's bracket, restated in numpy (DESIGN.md §5 "int8
prefilter"; the device side is vs_q8.hip + select_q8_kernel, checked on the
GPU by tools/q8_check.hip and tests/test_q8_gpu.py).

For rows x (bf16 values, or fp32), one collection scale S = max|x| / 127 and
x8 = clamp(rint(x / S), -127, 127); per 32-row tile dt = max |x - S x8| and
nt = max |x| rounded up; per query q, sq = max|q| / 127, q8, a = |sq q8|,
c = |q - sq q8| (rounded up) and sigma = (4 D + 64) 2^-24 |q|. Then for every
row, with m = a dt + c nt and the int32 dot q8 . x8:
    L = sqS dot - m - sigma nt  <=  s  <=  U = sqS dot + m + sigma nt
for any fp32 evaluation s of q . x. This file checks that on random,
clipped and adversarial rows against fp32 sums in several orders.
"""
import numpy as np
import pytest

D = 768


def _up(v):
    return np.nextafter(np.float32(v), np.float32(np.inf))


def _quantize_rows(X, S):
    X8 = np.clip(np.rint(X / S), -127, 127).astype(np.int32)
    d = X.astype(np.float64) - np.float64(S) * X8
    dn = np.sqrt((d * d).sum(1)) * (1 + 2.0 ** -30)
    xn = np.sqrt((X.astype(np.float64) ** 2).sum(1)) * (1 + 2.0 ** -30)
    dt = np.array([_up(dn[i:i + 32].max()) for i in range(0, len(X), 32)], np.float32)
    nt = np.array([_up(xn[i:i + 32].max()) for i in range(0, len(X), 32)], np.float32)
    return X8, dt, nt


def _quantize_query(q, S):
    amax = np.float32(np.abs(q).max())
    sq = np.float32(amax / np.float32(127)) if amax > 0 else np.float32(0)
    q8 = np.clip(np.rint(q / sq), -127, 127).astype(np.int32) if sq > 0 else np.zeros(D, np.int32)
    s = np.float64(sq) * q8
    a = _up(np.sqrt((s * s).sum()) * (1 + 2.0 ** -30))
    e = q.astype(np.float64) - s
    c = _up(np.sqrt((e * e).sum()) * (1 + 2.0 ** -30))
    nq = _up(np.sqrt((q.astype(np.float64) ** 2).sum()) * (1 + 2.0 ** -30))
    sigma = np.float32((4.0 * D + 64.0) * 2.0 ** -24 * float(nq) * (1 + 2.0 ** -20))
    return q8, np.float32(sq * np.float32(S)), a, c, sigma


def _fp32_sums(X, q):
    """fp32 scores in three orders: sequential, pairwise (numpy), reversed."""
    xf, qf = X.astype(np.float32), q.astype(np.float32)
    seq = np.zeros(len(X), np.float32)
    rev = np.zeros(len(X), np.float32)
    for i in range(D):
        seq = np.float32(seq + xf[:, i] * qf[i])
        rev = np.float32(rev + xf[:, D - 1 - i] * qf[D - 1 - i])
    return [seq, rev, (xf @ qf).astype(np.float32)]


def _bf16(a):
    u = np.ascontiguousarray(a, np.float32).view(np.uint32)
    u = (u + 0x7FFF + ((u >> 16) & 1)) & 0xFFFF0000
    return u.view(np.float32)


@pytest.mark.parametrize("case", ["unit_bf16", "fp32", "clipped", "spiky"])
def test_int8_bracket_holds(case):
    rng = np.random.default_rng(["unit_bf16", "fp32", "clipped", "spiky"].index(case) + 11)
    n = 1024
    X = rng.standard_normal((n, D)).astype(np.float32)
    X /= np.linalg.norm(X, axis=1, keepdims=True)
    if case == "unit_bf16":
        X = _bf16(X)
    S = np.float32(np.float32(np.abs(X).max()) / np.float32(127))
    if case == "clipped":  # rows written after S was chosen, 4x larger: clipped
        X[::7] *= 4
    if case == "spiky":  # one large coordinate per row, the rest tiny
        X[:, 5] = 0.9
        X[:, 6:] *= 0.01
        S = np.float32(np.float32(np.abs(X).max()) / np.float32(127))
    X8, dt, nt = _quantize_rows(X, S)
    for j in range(6):
        q = rng.standard_normal(D).astype(np.float32)
        q = _bf16(q / np.linalg.norm(q)) if case == "unit_bf16" else q / np.linalg.norm(q)
        if j == 5:
            q = q * np.float32(30.0)  # large norm
        q8, sqS, a, c, sigma = _quantize_query(q, S)
        dot = X8 @ q8  # exact in int64
        assert np.abs(dot).max() < 2 ** 24  # exact in fp32 too
        tile = np.arange(n) // 32
        m = a * dt[tile] + c * nt[tile]
        L = np.float32(dot.astype(np.float32) * sqS) - m - sigma * nt[tile]
        U = np.float32(dot.astype(np.float32) * sqS) + m + sigma * nt[tile]
        exact = X.astype(np.float64) @ q.astype(np.float64)
        assert np.all(L <= exact) and np.all(exact <= U), case
        for s in _fp32_sums(X, q):
            assert np.all(L <= s) and np.all(s <= U), case


def test_int8_window_is_narrow():
    """The bracket is worth having: for unit 768-d rows its width 2m is a
    fraction of the score spread (the int8 pass admits ~5x the rows the
    bf16 pass does, not all of them)."""
    rng = np.random.default_rng(3)
    X = rng.standard_normal((4096, D)).astype(np.float32)
    X = _bf16(X / np.linalg.norm(X, axis=1, keepdims=True))
    S = np.float32(np.float32(np.abs(X).max()) / np.float32(127))
    X8, dt, nt = _quantize_rows(X, S)
    q = _bf16(rng.standard_normal(D).astype(np.float32))
    q = _bf16(q / np.linalg.norm(q))
    q8, sqS, a, c, sigma = _quantize_query(q, S)
    m = float(a * dt.max() + c * nt.max())
    spread = float(np.std(X.astype(np.float64) @ q.astype(np.float64)))
    assert 0.2 < 2 * m / spread < 1.5, (m, spread)
