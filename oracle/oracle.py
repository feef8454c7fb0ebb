"""CPU oracle for the exact top-k search path — TEST INFRASTRUCTURE ONLY.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg
may import this module, and only as the checker / the timed CPU baseline.
The product (the package's C-ABI library) never calls it.

Two independent restatements of the reference path live here:

* ``liboracle.so`` (vsearch_oracle.c) — the primary oracle, C + OpenMP.
* ``np_*`` functions — a numpy restatement used to cross-check the C one.

Reference semantics restated (see vsearch_oracle.c for the full citation):
rag/vector-service/main.go:249-254 (Points.Search, Limit=top_k, no filter),
main.go:102-112 (Cosine collections, f32 storage), Qdrant
``CosineMetric::preprocess`` (upstream lib/segment/src/spaces/simple.rs,
unpinned ``qdrant/qdrant:latest``, docker-compose.yml:5).

Parity pinning: the reference ships no tests, fixtures or embeddings for this
path: parity is *unpinned by reference data*; the oracle
is pinned by analytic known-answer tests and C-vs-numpy agreement.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")
LIB512_PATH = os.path.join(HERE, "liboracle_avx512.so")  # CPU baseline on AVX-512 hosts

SEED_CORPUS = 0x5EED
SEED_QUERY = 0xC0FFEE

_lib = None


def build() -> str:
    """Compile liboracle.so (gcc, OpenMP) if missing or stale."""
    src = os.path.join(HERE, "vsearch_oracle.c")
    stale = [p for p in (LIB_PATH, LIB512_PATH)
             if not os.path.exists(p) or os.path.getmtime(p) < os.path.getmtime(src)]
    if stale:
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = ctypes.CDLL(LIB_PATH)
        u64, u32, i32 = ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        vp = ctypes.c_void_p
        L.oracle_generate.argtypes = [u64, u64, u64, u32, i32, vp]
        L.oracle_generate_raw.argtypes = [u64, u64, u64, u32, i32, vp]
        L.oracle_preprocess.argtypes = [vp, u64, u32, i32, i32, vp]
        L.oracle_search.argtypes = [vp, u64, u32, vp, u32, u32, u64, vp, vp, vp, vp]
        L.oracle_rescore.argtypes = [vp, u32, vp, u32, u32, vp, vp, u64, vp]
        L.oracle_cpu_scan.argtypes = [vp, i32, u64, u32, vp, u32, u32, i32, vp, vp]
        L.oracle_cpu_scan.restype = i32
        L.oracle_f32_to_bf16.argtypes = [ctypes.c_float]
        L.oracle_f32_to_bf16.restype = ctypes.c_uint16
        L.oracle_search_generated.argtypes = [u64, u64, u64, u32, i32, vp, u32, u32, i32, vp,
                                              vp, vp]
        L.oracle_rescore_generated.argtypes = [u64, u32, i32, vp, u32, u32, vp, vp, vp]
        L.oracle_checksum.argtypes = [vp, u64]
        L.oracle_checksum.restype = u64
        _lib = L
    return _lib


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------
# C oracle wrappers
# --------------------------------------------------------------------------
def generate(seed: int, grow0: int, n: int, dim: int, bf16: bool = False) -> np.ndarray:
    out = np.empty((n, dim), np.float32)
    lib().oracle_generate(seed, grow0, n, dim, int(bf16), _p(out))
    return out


def generate_raw(seed: int, grow0: int, n: int, dim: int, bf16: bool) -> np.ndarray:
    out = np.empty((n, dim), np.uint16 if bf16 else np.float32)
    lib().oracle_generate_raw(seed, grow0, n, dim, int(bf16), _p(out))
    return out


def preprocess(x: np.ndarray, cosine: bool, bf16: bool = False) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    out = np.empty_like(x)
    lib().oracle_preprocess(_p(x), x.shape[0], x.shape[1], int(cosine), int(bf16), _p(out))
    return out


def search(X: np.ndarray, Q: np.ndarray, k: int, row_base: int = 0):
    """Exact top-k of preprocessed queries Q against stored rows X.

    Returns (scores_f32, scores_f64, rows, counts)."""
    X = np.ascontiguousarray(X, np.float32)
    Q = np.ascontiguousarray(Q, np.float32)
    nq, dim = Q.shape
    s32 = np.zeros((nq, k), np.float32)
    s64 = np.zeros((nq, k), np.float64)
    rows = np.zeros((nq, k), np.uint64)
    cnt = np.zeros(nq, np.uint32)
    lib().oracle_search(_p(X), X.shape[0], dim, _p(Q), nq, k, row_base, _p(s32), _p(s64),
                        _p(rows), _p(cnt))
    return s32, s64, rows, cnt


def search_generated(seed: int, grow0: int, n: int, Q: np.ndarray, k: int, bf16: bool,
                     threads: int = 0):
    """Exact top-k over generator rows grow0 .. grow0+n-1 (a vs_generate corpus)
    without materialising it: rows are regenerated per thread block.

    Returns (scores_f64, rows, counts); rows are global row numbers."""
    Q = np.ascontiguousarray(Q, np.float32)
    nq, dim = Q.shape
    s64 = np.zeros((nq, k), np.float64)
    rows = np.zeros((nq, k), np.uint64)
    cnt = np.zeros(nq, np.uint32)
    lib().oracle_search_generated(seed, grow0, n, dim, int(bf16), _p(Q), nq, k, threads,
                                  _p(s64), _p(rows), _p(cnt))
    return s64, rows, cnt


def rescore_generated(seed: int, Q: np.ndarray, rows: np.ndarray, counts: np.ndarray,
                      bf16: bool) -> np.ndarray:
    """Exact fp64 scores of (query, global row) pairs of a generated corpus."""
    Q = np.ascontiguousarray(Q, np.float32)
    rows = np.ascontiguousarray(rows, np.uint64)
    counts = np.ascontiguousarray(counts, np.uint32)
    nq, k = rows.shape
    out = np.zeros((nq, k), np.float64)
    lib().oracle_rescore_generated(seed, Q.shape[1], int(bf16), _p(Q), nq, k, _p(rows),
                                   _p(counts), _p(out))
    return out


def rescore(X: np.ndarray, Q: np.ndarray, rows: np.ndarray, counts: np.ndarray,
            row_base: int = 0) -> np.ndarray:
    """Exact fp64 scores of the (query, row) pairs a device returned."""
    X = np.ascontiguousarray(X, np.float32)
    Q = np.ascontiguousarray(Q, np.float32)
    rows = np.ascontiguousarray(rows, np.uint64)
    counts = np.ascontiguousarray(counts, np.uint32)
    nq, k = rows.shape
    out = np.zeros((nq, k), np.float64)
    lib().oracle_rescore(_p(X), X.shape[1], _p(Q), nq, k, _p(rows), _p(counts), row_base,
                         _p(out))
    return out


def cpu_info() -> dict:
    """Host CPU model and whether it has AVX-512 (Linux /proc/cpuinfo)."""
    model, flags = "unknown", set()
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name") and model == "unknown":
                    model = line.split(":", 1)[1].strip()
                elif line.startswith("flags") and not flags:
                    flags = set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return {"model": model, "avx512": "avx512f" in flags, "logical_cpus": os.cpu_count()}


_scan_lib = None


def scan_lib():
    """The CPU-baseline build for this host: AVX-512 when the CPU has it."""
    global _scan_lib
    if _scan_lib is None:
        build()
        path = LIB512_PATH if cpu_info()["avx512"] and os.path.exists(LIB512_PATH) else LIB_PATH
        L = ctypes.CDLL(path)
        vp, u64, u32, i32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
        L.oracle_cpu_scan.argtypes = [vp, i32, u64, u32, vp, u32, u32, i32, vp, vp]
        L.oracle_cpu_scan.restype = i32
        L.oracle_cpu_scan_lanes.restype = i32
        _scan_lib = L
    return _scan_lib


def cpu_scan_isa() -> str:
    return "avx512" if scan_lib().oracle_cpu_scan_lanes() == 16 else "avx2"


def cpu_scan(X_raw: np.ndarray, bf16: bool, Q: np.ndarray, k: int, threads: int = 0):
    """Qdrant-style fp32 exact scan (the CPU baseline), one query at a time.
    Returns (scores, rows, threads)."""
    Q = np.ascontiguousarray(Q, np.float32)
    nq, dim = Q.shape
    s = np.zeros((nq, k), np.float32)
    r = np.zeros((nq, k), np.uint64)
    nth = scan_lib().oracle_cpu_scan(_p(X_raw), int(bf16), X_raw.shape[0], dim, _p(Q), nq, k,
                                     threads, _p(s), _p(r))
    return s, r, nth


# --------------------------------------------------------------------------
# independent numpy restatement (cross-check of the C oracle)
def checksum(data: bytes) -> int:
    """Snapshot data checksum (C restatement, vsearch_oracle.c oracle_checksum)."""
    buf = ctypes.create_string_buffer(bytes(data), len(data))
    return int(lib().oracle_checksum(buf, len(data)))


# --------------------------------------------------------------------------
_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _np_splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        x = x + np.uint64(0x9E3779B97F4A7C15)
        x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return x ^ (x >> np.uint64(31))


def np_gen_ints(seed: int, grow0: int, n: int, dim: int) -> np.ndarray:
    rows = np.arange(grow0, grow0 + n, dtype=np.uint64)
    with np.errstate(over="ignore"):
        rk = _np_splitmix64(np.uint64(seed) ^ (rows * np.uint64(0xD1B54A32D192ED03)))
        h = _np_splitmix64(rk[:, None] + np.arange(dim, dtype=np.uint64)[None, :])
    m = np.uint64(0xFFFF)
    s = (h & m) + ((h >> np.uint64(16)) & m) + ((h >> np.uint64(32)) & m) + (h >> np.uint64(48))
    return s.astype(np.int64) - 131070


def np_bf16_round(x: np.ndarray) -> np.ndarray:
    u = np.ascontiguousarray(x, np.float32).view(np.uint32).astype(np.uint64)
    nan = ((u & 0x7F800000) == 0x7F800000) & ((u & 0x007FFFFF) != 0)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) & 0xFFFF
    r = np.where(nan, (u >> 16) | 0x40, r).astype(np.uint32) << 16
    return r.view(np.float32)


def np_generate(seed: int, grow0: int, n: int, dim: int, bf16: bool = False) -> np.ndarray:
    m = np_gen_ints(seed, grow0, n, dim)
    s = (m * m).sum(axis=1)  # exact in int64
    nrm = np.sqrt(s.astype(np.float64))
    with np.errstate(invalid="ignore", divide="ignore"):
        y = np.where(s[:, None] > 0, m.astype(np.float64) / nrm[:, None], 0.0).astype(np.float32)
    return np_bf16_round(y) if bf16 else y


def np_sqnorm(x: np.ndarray) -> np.ndarray:
    n, dim = x.shape
    J = (dim + 63) // 64
    pad = np.zeros((n, J * 64), np.float64)
    pad[:, :dim] = x.astype(np.float64)
    v = pad.reshape(n, J, 64)
    lanes = np.zeros((n, 64), np.float64)
    for j in range(J):  # sequential per lane, as the device
        lanes = lanes + v[:, j, :] * v[:, j, :]
    idx = np.arange(64)
    for m in (32, 16, 8, 4, 2, 1):
        lanes = lanes + lanes[:, idx ^ m]
    return lanes[:, 0]


def np_preprocess(x: np.ndarray, cosine: bool, bf16: bool = False) -> np.ndarray:
    x = np.ascontiguousarray(x, np.float32)
    s = np_sqnorm(x)
    keep = (~np.bool_(cosine)) | (s < 1.1920928955078125e-07) | (np.abs(s - 1.0) <= 1.0e-6)
    with np.errstate(invalid="ignore", divide="ignore"):
        y = np.where(keep[:, None], x,
                     (x.astype(np.float64) / np.sqrt(s)[:, None]).astype(np.float32))
    y = y.astype(np.float32)
    return np_bf16_round(y) if bf16 else y


def np_search(X: np.ndarray, Q: np.ndarray, k: int, row_base: int = 0):
    """Exact top-k by fp64 scores; ties by row ascending. Returns (scores64, rows)."""
    S = Q.astype(np.float64) @ X.astype(np.float64).T  # (nq, n)
    n = X.shape[0]
    kk = min(k, n)
    rows = np.zeros((Q.shape[0], k), np.uint64)
    scores = np.zeros((Q.shape[0], k), np.float64)
    ar = np.arange(n)
    for i in range(Q.shape[0]):
        order = np.lexsort((ar, -S[i]))[:kk]
        rows[i, :kk] = order + row_base
        scores[i, :kk] = S[i, order]
    return scores, rows


# --------------------------------------------------------------------------
# parity rule of BASELINE.json north_star
# --------------------------------------------------------------------------
def check_topk(dev_scores, dev_rows, dev_count, ref_s64, ref_rows, ref_count, rescored,
               score_rtol: float, tie_rtol: float = 1e-5, atol: float = 1e-6):
    """Returns a list of human-readable violations (empty = parity).

    * counts must match;
    * every device score must equal the exact (fp64) score of the row it names
      within ``score_rtol`` relative (plus ``atol`` for scores near zero; unit
      vectors, so 1e-6 absolute is below one fp32 ulp of a dot of 768 terms);
    * at every rank j the device row must equal the oracle row, unless the
      oracle's exact scores of the two rows differ by less than ``tie_rtol``
      relative (a near-tie), in which case the device row must still be one the
      oracle ranks within the near-tie band of position j.
    """
    bad = []
    nq = len(ref_count)
    for i in range(nq):
        if int(dev_count[i]) != int(ref_count[i]):
            bad.append(f"q{i}: count {dev_count[i]} != {ref_count[i]}")
            continue
        c = int(ref_count[i])
        kth = ref_s64[i, c - 1] if c else 0.0
        for j in range(c):
            ex = rescored[i, j]
            tol = score_rtol * abs(ex) + atol
            if abs(float(dev_scores[i, j]) - ex) > tol:
                bad.append(f"q{i} r{j}: score {dev_scores[i, j]!r} vs exact {ex!r}")
            if int(dev_rows[i, j]) != int(ref_rows[i, j]):
                a = ref_s64[i, j]
                band = tie_rtol * abs(a) + atol
                # the device row must be an exact-score near-tie of the oracle's row,
                # and must not fall below the oracle's k-th score by more than the band
                if abs(ex - a) > band or ex < kth - (tie_rtol * abs(kth) + atol):
                    bad.append(f"q{i} r{j}: row {dev_rows[i, j]} (exact {ex!r}) != "
                               f"oracle row {ref_rows[i, j]} ({a!r})")
        if c and len(set(int(x) for x in dev_rows[i, :c])) != c:
            bad.append(f"q{i}: duplicate rows returned")
    return bad


def np_checksum(data: bytes) -> int:
    """numpy restatement of the snapshot checksum (vectorised over words)."""
    b = bytes(data)
    b += b"\0" * (-len(b) % 8)
    w = np.frombuffer(b, dtype="<u8").astype(np.uint64)
    with np.errstate(over="ignore"):
        i = np.arange(w.size, dtype=np.uint64)
        h = _np_splitmix64(w ^ (i * np.uint64(0x9E3779B97F4A7C15)))
        return int(np.sum(h, dtype=np.uint64))
