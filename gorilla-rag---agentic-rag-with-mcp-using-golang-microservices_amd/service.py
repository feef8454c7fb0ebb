"""ctypes binding of the vector-service handler mirror (include/vsearch_service.h).

``VectorService.handle(method, path, body)`` answers exactly what
rag/vector-service's Go handlers answer (main.go:121-278): same routes, JSON
shapes, status codes and messages, with the HIP engine in place of Qdrant.
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import Optional, Tuple

from .engine import HERE, VSError, _check, load_library

SVC_LIB_PATH = os.path.join(HERE, "lib", "libvsearch_service.so")

_svc = None


def load_service_library(path: str = SVC_LIB_PATH):
    global _svc
    if _svc is not None:
        return _svc
    load_library()  # resolves libvsearch.so first (same directory)
    if not os.path.exists(path):
        raise ImportError(f"{path} is missing: run __graft_entry__.build()")
    L = ctypes.CDLL(path)
    vp, cp, sz = ctypes.c_void_p, ctypes.c_char_p, ctypes.c_size_t
    L.vsvc_open.argtypes = [vp, cp, ctypes.POINTER(vp)]
    L.vsvc_open.restype = ctypes.c_int
    L.vsvc_close.argtypes = [vp]
    L.vsvc_close.restype = None
    L.vsvc_handle.argtypes = [vp, cp, cp, cp, sz, ctypes.POINTER(ctypes.c_int),
                              ctypes.POINTER(vp), ctypes.POINTER(sz), ctypes.POINTER(cp)]
    L.vsvc_handle.restype = ctypes.c_int
    L.vsvc_free.argtypes = [vp]
    L.vsvc_free.restype = None
    L.vsvc_reencode.argtypes = [cp, sz, ctypes.POINTER(vp)]
    L.vsvc_reencode.restype = ctypes.c_int
    L.vsvc_validate.argtypes = [cp, cp, sz, ctypes.POINTER(vp)]
    L.vsvc_validate.restype = ctypes.c_int
    L.vsvc_bulk_generate.argtypes = [vp, cp, ctypes.c_uint64, ctypes.c_uint64]
    L.vsvc_bulk_generate.restype = ctypes.c_int
    L.vsvc_point_id.argtypes = [vp, cp, ctypes.c_uint64, cp, sz]
    L.vsvc_point_id.restype = ctypes.c_int
    L.vsvc_snapshot.argtypes = [vp, cp]
    L.vsvc_snapshot.restype = ctypes.c_int
    L.vsvc_restore.argtypes = [vp, cp]
    L.vsvc_restore.restype = ctypes.c_int
    L.vsvc_stats.argtypes = [vp, ctypes.POINTER(vp)]
    L.vsvc_stats.restype = ctypes.c_int
    L.vsvc_loadgen.argtypes = [vp, cp, ctypes.POINTER(vp)]
    L.vsvc_loadgen.restype = ctypes.c_int
    L.vsvc_http_start.argtypes = [vp, cp, ctypes.POINTER(vp)]
    L.vsvc_http_start.restype = ctypes.c_int
    L.vsvc_http_port.argtypes = [vp]
    L.vsvc_http_port.restype = ctypes.c_int
    L.vsvc_http_stop.argtypes = [vp]
    L.vsvc_http_stop.restype = None
    _svc = L
    return L


def _take(L, p: ctypes.c_void_p, n: Optional[int] = None) -> bytes:
    if not p.value:
        return b""
    data = ctypes.string_at(p.value, n) if n is not None else ctypes.string_at(p.value)
    L.vsvc_free(p)
    return data


def reencode(doc: bytes) -> Tuple[int, bytes]:
    """(0, Go json.Encoder output) or (-1, syntax error text)."""
    L = load_service_library()
    out = ctypes.c_void_p()
    rc = L.vsvc_reencode(doc, len(doc), ctypes.byref(out))
    return rc, _take(L, out)


def validate(path: str, body: bytes) -> Tuple[int, str]:
    """(400, decode error) or (0, '') for a /search or /upsert body."""
    L = load_service_library()
    out = ctypes.c_void_p()
    rc = L.vsvc_validate(path.encode(), body, len(body), ctypes.byref(out))
    return rc, _take(L, out).decode()


class VectorService:
    """rag/vector-service's four handlers over an engine (not owned)."""

    def __init__(self, engine, config: Optional[dict] = None):
        L = load_service_library()
        h = ctypes.c_void_p()
        cfg = json.dumps(config).encode() if config is not None else None
        rc = L.vsvc_open(engine.handle, cfg, ctypes.byref(h))
        if rc != 0:
            _check(rc)
        self._h, self._L, self.engine = h, L, engine

    def close(self):
        if getattr(self, "_h", None):
            self._L.vsvc_close(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def handle(self, method: str, path: str, body: bytes = b"") -> Tuple[int, bytes, str]:
        st = ctypes.c_int()
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        ct = ctypes.c_char_p()
        rc = self._L.vsvc_handle(self._h, method.encode(), path.encode(), body, len(body),
                                 ctypes.byref(st), ctypes.byref(out), ctypes.byref(n),
                                 ctypes.byref(ct))
        if rc != 0:
            raise VSError(rc, "vsvc_handle failed")
        return st.value, _take(self._L, out, n.value), ct.value.decode()

    def bulk_generate(self, collection: str, n: int, seed: int) -> None:
        """n synthetic device-generated points with synthetic UUIDs (empty collection)."""
        _check(self._L.vsvc_bulk_generate(self._h, collection.encode(), n, seed))

    def snapshot(self, directory: str) -> None:
        """Save every collection (rows + UUIDs + payloads) under `directory`."""
        _check(self._L.vsvc_snapshot(self._h, os.fsencode(directory)))

    def restore(self, directory: str) -> None:
        """Load the collections saved under `directory` (service still empty)."""
        _check(self._L.vsvc_restore(self._h, os.fsencode(directory)))

    def point_id(self, collection: str, row: int) -> str:
        buf = ctypes.create_string_buffer(40)
        _check(self._L.vsvc_point_id(self._h, collection.encode(), row, buf, 40))
        return buf.value.decode()

    def stats(self) -> dict:
        """Batcher counters (vsvc_stats)."""
        out = ctypes.c_void_p()
        _check(self._L.vsvc_stats(self._h, ctypes.byref(out)))
        return json.loads(_take(self._L, out))

    def loadgen(self, collections, dim: int, clients: int = 16, seconds: float = 5.0,
                k_min: int = 3, k_max: int = 50, queries: int = 256, seed: int = 1,
                http: Optional[str] = None, keepalive: bool = True) -> dict:
        """Closed-loop /search load (vsvc_loadgen): retrieval-service-shaped
        requests from `clients` threads for `seconds`; returns QPS + latency.
        `http="host:port"` posts them over TCP to a listener instead."""
        spec = {"collections": list(collections), "dim": dim, "clients": clients,
                "seconds": seconds, "k_min": k_min, "k_max": k_max, "queries": queries,
                "seed": seed}
        if http is not None:
            spec.update(http=http, keepalive=keepalive)
        out = ctypes.c_void_p()
        _check(self._L.vsvc_loadgen(self._h, json.dumps(spec).encode(), ctypes.byref(out)))
        return json.loads(_take(self._L, out))

    def serve(self, addr: str = "127.0.0.1:0") -> "HttpListener":
        """HTTP/1.1 listener on `addr` in front of the handlers (vsvc_http_start)."""
        h = ctypes.c_void_p()
        _check(self._L.vsvc_http_start(self._h, addr.encode(), ctypes.byref(h)))
        return HttpListener(self._L, h)


class HttpListener:
    """A running vsvc_http listener; stop() before closing the service."""

    def __init__(self, L, h):
        self._L, self._h = L, h
        self.port = L.vsvc_http_port(h)

    def stop(self):
        if self._h:
            self._L.vsvc_http_stop(self._h)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.stop()
