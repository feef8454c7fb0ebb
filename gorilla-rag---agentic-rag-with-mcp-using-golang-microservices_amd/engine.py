"""ctypes binding of the engine's C-ABI (include/vsearch.h).

This is the Python counterpart of the cgo package shown in INTEGRATION.md:
the same entry points, the same ownership rules (caller-owned buffers, no
retained pointers), and errors surfaced as exceptions carrying the
``vs_status`` code and ``vs_last_error()`` text.

There is no CPU fallback anywhere in this module: when the HIP library is
missing or no GPU is visible, the calls fail loudly.
"""
from __future__ import annotations

import ctypes
import os
from typing import Optional, Sequence, Tuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "lib", "libvsearch.so")

VS_OK = 0
VS_ERR_INVALID_ARG = -1
VS_ERR_NOT_FOUND = -2
VS_ERR_DIM_MISMATCH = -3
VS_ERR_OOM = -4
VS_ERR_DEVICE = -5
VS_ERR_EXISTS = -6
VS_ERR_INTERNAL = -7
VS_ERR_IO = -8

METRIC_COSINE = 0
METRIC_DOT = 1
DTYPE_F32 = 0
DTYPE_BF16 = 1
FLAG_TIMING = 1
FLAG_TIMING_MERGE = 2
FLAG_TIMING_SAMPLE = 4
FLAG_PLACE_COLLECTIONS = 8
FLAG_ENGINE_PER_SHARD = 16
FLAG_NO_PREFILTER = 32
FLAG_NO_SPECULATIVE = 64

# Every function include/vsearch.h declares (checked by tests/test_abi.py).
EXPORTS = (
    "vs_open", "vs_close", "vs_device_count", "vs_collection_create",
    "vs_collection_info", "vs_collection_drop", "vs_upsert", "vs_generate",
    "vs_generate_vectors",
    "vs_read_rows", "vs_search", "vs_search_keys", "vs_merge_keys",
    "vs_decode_keys", "vs_health", "vs_last_error", "vs_timing",
    "vs_snapshot", "vs_restore", "vs_checksum", "vs_search_filtered",
    "vs_filter_create", "vs_filter_drop", "vs_search_filter_id", "vs_open_multi",
    "vs_engine_layout", "vs_comm_unique_id", "vs_comm_init", "vs_gather_merge_keys",
    "vs_copy_last_error", "vs_build_id", "vs_collection_placement", "vs_runtime_check",
    "vs_collection_prefilter_bytes", "vs_collection_spec_stats",
)
COMM_ID_BYTES = 128


class VSError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"vsearch error {code}: {msg}")
        self.code = code
        self.msg = msg


class _Config(ctypes.Structure):
    _fields_ = [("device", ctypes.c_int32), ("flags", ctypes.c_uint32)]


class _ConfigMulti(ctypes.Structure):
    _fields_ = [("devices", ctypes.POINTER(ctypes.c_int32)), ("n_shards", ctypes.c_uint32),
                ("flags", ctypes.c_uint32)]


_lib = None


def _torch_runtime_first():
    """Imports torch (when installed) before libvsearch is loaded, so the
    process holds ONE HIP runtime. torch's ROCm wheel bundles its own
    libamdhip64.so and links it by file name; libvsearch links
    libamdhip64.so.7 by soname. torch first: libvsearch binds to the runtime
    torch loaded (same soname). libvsearch first: a later torch import maps a
    second runtime, whose null stream and queues are unordered with ours --
    a vs_search_keys on torch's stream then races torch's own work (the
    round-3 driver failure). VS_TORCH_FIRST=0 skips this."""
    if os.environ.get("VS_TORCH_FIRST", "1") == "0":
        return
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


def hip_runtimes() -> list:
    """Paths of the libamdhip64 runtimes mapped into this process."""
    out = []
    try:
        with open("/proc/self/maps") as f:
            for line in f:
                p = line.split()[-1] if len(line.split()) >= 6 else ""
                if os.path.basename(p).startswith("libamdhip64.so") and p not in out:
                    out.append(p)
    except OSError:
        pass
    return out


def load_library(path: str = LIB_PATH):
    """Loads libvsearch.so (built by __graft_entry__.build()). Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: build the HIP library first "
                          "(python -c 'import __graft_entry__ as g; g.build()')")
    _torch_runtime_first()
    L = ctypes.CDLL(path)
    vp, u32, u64, i32 = ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint64, ctypes.c_int
    cp = ctypes.c_char_p
    sig = {
        "vs_open": ([ctypes.POINTER(_Config), ctypes.POINTER(vp)], i32),
        "vs_open_multi": ([ctypes.POINTER(_ConfigMulti), ctypes.POINTER(vp)], i32),
        "vs_engine_layout": ([vp, vp, vp], i32),
        "vs_collection_placement": ([vp, cp, vp], i32),
        "vs_collection_prefilter_bytes": ([vp, cp, vp], i32),
        "vs_collection_spec_stats": ([vp, cp, vp], i32),
        "vs_close": ([vp], None),
        "vs_device_count": ([], i32),
        "vs_collection_create": ([vp, cp, u32, i32, i32, u64, u64], i32),
        "vs_collection_info": ([vp, cp, vp, vp, vp, vp], i32),
        "vs_collection_drop": ([vp, cp], i32),
        "vs_upsert": ([vp, cp, u64, u32, vp, vp], i32),
        "vs_generate": ([vp, cp, u64, u64], i32),
        "vs_generate_vectors": ([vp, u64, u64, u64, u32, vp, vp], i32),
        "vs_read_rows": ([vp, cp, u64, u64, vp], i32),
        "vs_search": ([vp, cp, vp, u32, u32, u32, vp, vp, vp], i32),
        "vs_search_keys": ([vp, cp, vp, u32, u32, u32, vp, vp], i32),
        "vs_merge_keys": ([vp, vp, u32, u32, u32, u32, vp, vp], i32),
        "vs_comm_unique_id": ([vp], i32),
        "vs_comm_init": ([vp, u32, u32, vp], i32),
        "vs_gather_merge_keys": ([vp, vp, u32, u32, u32, vp, vp], i32),
        "vs_decode_keys": ([vp, vp, u32, u32, vp, vp, vp, vp], i32),
        "vs_health": ([vp, ctypes.c_char_p, ctypes.c_size_t], i32),
        "vs_last_error": ([], ctypes.c_char_p),
        "vs_copy_last_error": ([ctypes.c_char_p, ctypes.c_size_t], ctypes.c_size_t),
        "vs_build_id": ([], ctypes.c_char_p),
        "vs_runtime_check": ([], i32),
        "vs_timing": ([vp, vp, vp, vp, vp, i32], i32),
        "vs_snapshot": ([vp, cp, cp], i32),
        "vs_restore": ([vp, cp, cp], i32),
        "vs_checksum": ([vp, cp, ctypes.POINTER(u64)], i32),
        "vs_search_filtered": ([vp, cp, vp, u32, u32, u32, vp, u64, vp, vp, vp], i32),
        "vs_filter_create": ([vp, cp, vp, u64, vp], i32),
        "vs_filter_drop": ([vp, u64], i32),
        "vs_search_filter_id": ([vp, cp, vp, u32, u32, u32, u64, vp, vp, vp], i32),
    }
    for name, (args, res) in sig.items():
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    _lib = L
    return L


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _check(rc: int):
    if rc != VS_OK:
        msg = _lib.vs_last_error().decode("utf-8", "replace")
        raise VSError(rc, msg)


def pack_allow(mask: np.ndarray) -> np.ndarray:
    """bool per row -> uint64 words, bit r of word r // 64 (vs_search_filtered)."""
    m = np.asarray(mask, np.bool_).ravel()
    pad = np.zeros((-m.size) % 64, np.bool_)
    bits = np.packbits(np.concatenate([m, pad]), bitorder="little")
    return bits.view("<u8").astype(np.uint64) if bits.size else np.zeros(0, np.uint64)


def build_id() -> str:
    """vs_build_id() of the loaded library: build.py tree_hash() of its sources."""
    return load_library().vs_build_id().decode()


def device_count() -> int:
    return int(load_library().vs_device_count())


# key helpers (include/vsearch.h "Result key layout")
def keys_decode(keys: np.ndarray) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    keys = np.asarray(keys, np.uint64)
    o = (keys >> np.uint64(32)).astype(np.uint32)
    u = np.where(o & 0x80000000, o & 0x7FFFFFFF, ~o).astype(np.uint32)
    scores = u.view(np.float32).copy()
    rows = (np.uint32(0xFFFFFFFF) - (keys & np.uint64(0xFFFFFFFF)).astype(np.uint32)).astype(np.uint64)
    valid = keys != 0
    scores[~valid] = 0
    rows[~valid] = 0
    return scores, rows, valid.sum(axis=-1).astype(np.uint32)


class VectorEngine:
    """One engine handle (vs_open, or vs_open_multi when `shards` is given).
    Mirrors the C-ABI 1:1.

    ``shards``: HIP device ordinal of every shard (may repeat), e.g.
    ``[0, 1, 2, 3, 4, 5, 6, 7]`` for one shard per GPU of a node; collections
    are then row-striped over the shards and searched with one RCCL
    all-gather per call (include/vsearch.h "multi-GPU engine"), or with
    ``place_collections`` each placed whole on one device
    (VS_FLAG_PLACE_COLLECTIONS); ``engine_per_shard`` then gives every entry
    of ``shards`` its own device engine even where ordinals repeat
    (VS_FLAG_ENGINE_PER_SHARD). ``prefilter=False`` keeps no int8 copies
    (VS_FLAG_NO_PREFILTER: batched bf16 searches run the bf16 pass);
    ``speculative=False`` runs every int8 batch on its sample pass
    (VS_FLAG_NO_SPECULATIVE, DESIGN.md §5 "Speculative bound")."""

    def __init__(self, device: int = -1, timing: bool = False, timing_merge: bool = False,
                 timing_sample: bool = False, shards: Optional[Sequence[int]] = None,
                 place_collections: bool = False, engine_per_shard: bool = False,
                 prefilter: bool = True, speculative: bool = True):
        L = load_library()
        flags = ((FLAG_TIMING if timing else 0) |
                 (FLAG_TIMING_MERGE if timing and timing_merge else 0) |
                 (FLAG_TIMING_SAMPLE if timing and timing_sample else 0) |
                 (FLAG_PLACE_COLLECTIONS if place_collections else 0) |
                 (FLAG_ENGINE_PER_SHARD if engine_per_shard else 0) |
                 (0 if prefilter else FLAG_NO_PREFILTER) |
                 (0 if speculative else FLAG_NO_SPECULATIVE))
        h = ctypes.c_void_p()
        if shards is None:
            cfg = _Config(device, flags)
            _check(L.vs_open(ctypes.byref(cfg), ctypes.byref(h)))
        else:
            devs = (ctypes.c_int32 * len(shards))(*[int(x) for x in shards])
            cfgm = _ConfigMulti(devs, len(shards), flags)
            _check(L.vs_open_multi(ctypes.byref(cfgm), ctypes.byref(h)))
        self._h = h
        self._L = L

    def layout(self) -> Tuple[int, int]:
        """(shards, distinct devices) of this engine."""
        s, d = ctypes.c_uint32(), ctypes.c_uint32()
        _check(self._L.vs_engine_layout(self._h, ctypes.byref(s), ctypes.byref(d)))
        return s.value, d.value

    def placement(self, name: str) -> int:
        """HIP device holding the whole collection, or -1 when it is row-striped."""
        d = ctypes.c_int32()
        _check(self._L.vs_collection_placement(self._h, name.encode(), ctypes.byref(d)))
        return d.value


    def prefilter_bytes(self, name: str) -> int:
        """HBM bytes of the collection's int8 prefilter copy (0: none; its
        batched searches then run the bf16 pass). See VS_FLAG_NO_PREFILTER."""
        b = ctypes.c_uint64()
        _check(self._L.vs_collection_prefilter_bytes(self._h, name.encode(), ctypes.byref(b)))
        return int(b.value)

    def spec_stats(self, name: str) -> dict:
        """Counters of the collection's speculative bound (vs_collection_spec_stats,
        DESIGN.md §5): batches tried, of those failed (the sample path
        re-answered: the bench's `spec_fallbacks`), and batches a cool-down or
        an unset ratio sent to the sample path. Waits for the device."""
        a = (ctypes.c_uint64 * 4)()
        _check(self._L.vs_collection_spec_stats(self._h, name.encode(), a))
        return {"tries": int(a[0]), "fallbacks": int(a[1]), "skipped": int(a[2])}

    def close(self):
        if getattr(self, "_h", None):
            self._L.vs_close(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # collections ---------------------------------------------------------
    def create_collection(self, name: str, dim: int, metric: int = METRIC_COSINE,
                          dtype: int = DTYPE_F32, capacity: int = 0, row_base: int = 0):
        _check(self._L.vs_collection_create(self._h, name.encode(), dim, metric, dtype,
                                            capacity, row_base))

    def collection_info(self, name: str) -> dict:
        dim, rows = ctypes.c_uint32(), ctypes.c_uint64()
        metric, dtype = ctypes.c_int(), ctypes.c_int()
        _check(self._L.vs_collection_info(self._h, name.encode(), ctypes.byref(dim),
                                          ctypes.byref(rows), ctypes.byref(metric),
                                          ctypes.byref(dtype)))
        return {"dim": dim.value, "rows": rows.value, "metric": metric.value,
                "dtype": dtype.value}

    def drop_collection(self, name: str):
        _check(self._L.vs_collection_drop(self._h, name.encode()))

    # store side ----------------------------------------------------------
    def upsert(self, name: str, rows: Sequence[int], vectors: np.ndarray):
        v = np.ascontiguousarray(vectors, np.float32)
        r = np.ascontiguousarray(rows, np.uint64)
        if v.ndim != 2 or v.shape[0] != r.shape[0]:
            raise ValueError("vectors must be (n, dim) with one row number per vector")
        _check(self._L.vs_upsert(self._h, name.encode(), r.shape[0], v.shape[1], _p(r), _p(v)))

    def generate(self, name: str, n: int, seed: int):
        _check(self._L.vs_generate(self._h, name.encode(), n, seed))

    def generate_vectors(self, seed: int, row0: int, n: int, dim: int, d_out: int,
                         stream: int = 0):
        _check(self._L.vs_generate_vectors(self._h, seed, row0, n, dim, ctypes.c_void_p(d_out),
                                           ctypes.c_void_p(stream)))

    # snapshot / restore ---------------------------------
    def snapshot(self, name: str, path: str):
        """Write the collection's stored rows to `path` (vs_snapshot)."""
        _check(self._L.vs_snapshot(self._h, name.encode(), os.fsencode(path)))

    def restore(self, name: str, path: str):
        """Create collection `name` from a snapshot file (vs_restore)."""
        _check(self._L.vs_restore(self._h, name.encode(), os.fsencode(path)))

    def checksum(self, name: str) -> int:
        """Device checksum of the stored rows (vs_checksum)."""
        out = ctypes.c_uint64()
        _check(self._L.vs_checksum(self._h, name.encode(), ctypes.byref(out)))
        return out.value

    def read_rows(self, name: str, first: int, n: int) -> np.ndarray:
        dim = self.collection_info(name)["dim"]
        out = np.empty((n, dim), np.float32)
        _check(self._L.vs_read_rows(self._h, name.encode(), first, n, _p(out)))
        return out

    # search side ---------------------------------------------------------
    def search(self, name: str, queries: np.ndarray, k: int):
        q = np.ascontiguousarray(queries, np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        scores = np.zeros((nq, k), np.float32)
        rows = np.zeros((nq, k), np.uint64)
        count = np.zeros(nq, np.uint32)
        _check(self._L.vs_search(self._h, name.encode(), _p(q), nq, q.shape[1], k, _p(scores),
                                 _p(rows), _p(count)))
        return scores, rows, count

    def search_filtered(self, name: str, queries: np.ndarray, k: int, allow: np.ndarray):
        """search() restricted to the rows whose bit is set in `allow` (bool per
        local row, or packed uint64 words: bit r of word r // 64)."""
        q = np.ascontiguousarray(queries, np.float32)
        if q.ndim == 1:
            q = q[None, :]
        a = np.asarray(allow)
        if a.dtype == np.bool_:
            a = pack_allow(a)
        a = np.ascontiguousarray(a, np.uint64)
        nq = q.shape[0]
        scores = np.zeros((nq, k), np.float32)
        rows = np.zeros((nq, k), np.uint64)
        count = np.zeros(nq, np.uint32)
        _check(self._L.vs_search_filtered(self._h, name.encode(), _p(q), nq, q.shape[1], k,
                                          _p(a), a.size, _p(scores), _p(rows), _p(count)))
        return scores, rows, count

    def filter_create(self, name: str, allow: np.ndarray) -> int:
        """Uploads a filter bitmap (bool per row or packed words) once; returns
        its id for search_filter_id (vs_filter_create)."""
        a = np.asarray(allow)
        if a.dtype == np.bool_:
            a = pack_allow(a)
        a = np.ascontiguousarray(a, np.uint64)
        fid = ctypes.c_uint64()
        _check(self._L.vs_filter_create(self._h, name.encode(), _p(a), a.size,
                                        ctypes.byref(fid)))
        return fid.value

    def filter_drop(self, filter_id: int):
        _check(self._L.vs_filter_drop(self._h, filter_id))

    def search_filter_id(self, name: str, queries: np.ndarray, k: int, filter_id: int):
        q = np.ascontiguousarray(queries, np.float32)
        if q.ndim == 1:
            q = q[None, :]
        nq = q.shape[0]
        scores = np.zeros((nq, k), np.float32)
        rows = np.zeros((nq, k), np.uint64)
        count = np.zeros(nq, np.uint32)
        _check(self._L.vs_search_filter_id(self._h, name.encode(), _p(q), nq, q.shape[1], k,
                                           filter_id, _p(scores), _p(rows), _p(count)))
        return scores, rows, count

    def search_keys(self, name: str, d_queries: int, nq: int, dim: int, k: int, d_keys: int,
                    stream: int = 0):
        _check(self._L.vs_search_keys(self._h, name.encode(), ctypes.c_void_p(d_queries), nq,
                                      dim, k, ctypes.c_void_p(d_keys), ctypes.c_void_p(stream)))

    def merge_keys(self, d_lists: int, n_lists: int, nq: int, k_in: int, k: int,
                   d_out: int, stream: int = 0):
        _check(self._L.vs_merge_keys(self._h, ctypes.c_void_p(d_lists), n_lists, nq, k_in, k,
                                     ctypes.c_void_p(d_out), ctypes.c_void_p(stream)))

    # one process per GPU (include/vsearch.h "one process per GPU") -------
    @staticmethod
    def comm_unique_id() -> bytes:
        """A fresh RCCL unique id (made on one rank, handed to all)."""
        buf = ctypes.create_string_buffer(COMM_ID_BYTES)
        _check(load_library().vs_comm_unique_id(buf))
        return buf.raw

    def comm_init(self, n_ranks: int, rank: int, uid: bytes):
        """Joins the ranks' communicator (collective: every rank calls it)."""
        if len(uid) != COMM_ID_BYTES:
            raise ValueError(f"the unique id is {COMM_ID_BYTES} bytes")
        buf = ctypes.create_string_buffer(bytes(uid), COMM_ID_BYTES)
        _check(self._L.vs_comm_init(self._h, n_ranks, rank, buf))

    def gather_merge_keys(self, d_local: int, nq: int, k_in: int, k: int, d_out: int,
                          stream: int = 0):
        """All-gather of every rank's [nq][k_in] keys + merge to [nq][k], on `stream`."""
        _check(self._L.vs_gather_merge_keys(self._h, ctypes.c_void_p(d_local), nq, k_in, k,
                                            ctypes.c_void_p(d_out), ctypes.c_void_p(stream)))

    def decode_keys(self, d_keys: int, nq: int, k: int, stream: int = 0):
        scores = np.zeros((nq, k), np.float32)
        rows = np.zeros((nq, k), np.uint64)
        count = np.zeros(nq, np.uint32)
        _check(self._L.vs_decode_keys(self._h, ctypes.c_void_p(d_keys), nq, k, _p(scores),
                                      _p(rows), _p(count), ctypes.c_void_p(stream)))
        return scores, rows, count

    def health(self) -> str:
        buf = ctypes.create_string_buffer(1024)
        rc = self._L.vs_health(self._h, buf, len(buf))
        if rc not in (VS_OK, VS_ERR_DEVICE):
            _check(rc)
        return buf.value.decode()

    def timing(self, reset: bool = False) -> dict:
        sm, mm = ctypes.c_double(), ctypes.c_double()
        sn, mn = ctypes.c_uint64(), ctypes.c_uint64()
        _check(self._L.vs_timing(self._h, ctypes.byref(sm), ctypes.byref(sn),
                                 ctypes.byref(mm), ctypes.byref(mn), int(reset)))
        return {"scan_ms": sm.value, "scan_n": sn.value, "merge_ms": mm.value,
                "merge_n": mn.value}
