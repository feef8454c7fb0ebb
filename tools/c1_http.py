"""Config C1 (BASELINE.json configs[0]): the regulatory_docs collection
(~220 x 768 fp32 chunk embeddings, 2 ingested PDFs x ~110 chunks + 1) and a
single /search with top_k = 5, cosine, timed as the reference's callers see
it: over HTTP. SURVEY.md §8(d): "For C1, time the full HTTP /search on CPU
backend versus GPU backend".

    python tools/c1_http.py [--backend gpu|cpu|both] [--seconds 3]

Points go in through POST /upsert with ingest-service's body
(rag/ingest-service/main.go:359-386: id, vector, payload {text,
document_id, position}, ~500-rune texts); searches are retrieval-service's
body (rag/retrieval-service/main.go:221-226) posted by vsvc_loadgen's HTTP
client (C++, keep-alive) from 1 and 16 closed-loop clients, k fixed at 5.
The same service code (csrc/service: listener, handlers, batcher) runs over
  * gpu: the HIP engine (libvsearch.so) on cuda:0;
  * cpu: the engine C-ABI's CPU test double (tests/tsan/fake_engine.cpp: a
    brute-force exact scan under one reader/writer lock, test-only code,
    built here with g++ into a scratch library) -- the stand-in for the
    reference's CPU engine (Qdrant, not runnable here).
Embeddings are synthetic unit vectors (the Gemini vectors are not shipped).
One JSON line per (backend, clients).
"""
import argparse
import ctypes
import http.client
import json
import os
import subprocess
import sys
import tempfile
import uuid

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SVC = os.path.join(ROOT, "gorilla-rag---agentic-rag-with-mcp-using-golang-microservices_amd",
                   "csrc", "service")
N_DOCS, CHUNKS, DIM = 2, 110, 768


def _points(rng, doc, n):
    words = ["RBI", "shall", "merchant", "KYC", "payment", "aggregator", "settlement", "escrow",
             "account", "compliance", "directions", "regulated", "entity", "customer", "due",
             "diligence", "nodal", "bank", "report", "within"]
    pts = []
    for i in range(n):
        v = rng.standard_normal(DIM)
        text = " ".join(words[j] for j in rng.integers(0, len(words), 70))[:500]
        pts.append({"id": str(uuid.UUID(bytes=rng.bytes(16), version=4)),
                    "vector": [float(x) for x in (v / np.linalg.norm(v)).astype(np.float32)],
                    "payload": {"text": text, "document_id": doc, "position": i}})
    return pts


def _ingest(port, rng):
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=60)
    docs = [(f"doc-{d}", CHUNKS) for d in range(N_DOCS)] + [("test_doc", 1)]
    total = 0
    for doc, n in docs:
        body = json.dumps({"collection": "regulatory_docs", "points": _points(rng, doc, n)})
        c.request("POST", "/upsert", body=body, headers={"Content-Type": "application/json"})
        r = c.getresponse()
        out = r.read()
        if r.status != 200:
            raise RuntimeError(f"upsert failed: {r.status} {out[:200]!r}")
        total += n
    c.close()
    return total


def _measure(loadgen, port, backend, seconds):
    lines = []
    for clients in (1, 16):
        spec = {"collections": ["regulatory_docs"], "dim": DIM, "clients": clients,
                "seconds": 0.5, "k_min": 5, "k_max": 5, "http": f"127.0.0.1:{port}"}
        loadgen(spec)  # warm-up
        spec["seconds"] = seconds
        rep = loadgen(spec)
        lines.append({"workload": "C1: regulatory_docs 221 x 768 fp32 cosine, top_k 5, "
                                  "HTTP /search (keep-alive), closed loop",
                      "backend": backend, "clients": clients, "qps": round(rep["qps"], 1),
                      "lat_ms": {k: round(v, 4) for k, v in rep["lat_ms"].items()},
                      "requests": rep["requests"], "errors": rep["errors"],
                      "first_error": rep["first_error"][:200]})
        print(json.dumps(lines[-1]), flush=True)
    return lines


def run_gpu(seconds):
    import torch  # noqa: F401  (binds torch's HIP runtime first, as bench.py does)
    import __graft_entry__ as ge
    from importlib import import_module
    pkg = ge.load_package()
    svcmod = import_module(pkg.__name__ + ".service")
    eng = pkg.VectorEngine(device=0)
    svc = svcmod.VectorService(eng)  # reference defaults: 3 x 768 Cosine fp32
    try:
        with svc.serve("127.0.0.1:0") as lis:
            _ingest(lis.port, np.random.default_rng(7))

            def lg(spec):
                return svc.loadgen(spec["collections"], spec["dim"], clients=spec["clients"],
                                   seconds=spec["seconds"], k_min=5, k_max=5,
                                   http=spec["http"])
            return _measure(lg, lis.port, "gpu (HIP engine, MI355X)", seconds)
    finally:
        svc.close()
        eng.close()


def run_cpu(seconds):
    d = tempfile.mkdtemp(prefix="c1cpu")
    so = os.path.join(d, "libvsvc_cpu.so")
    srcs = [os.path.join(SVC, f) for f in ("json.cpp", "vector_service.cpp", "batcher.cpp",
                                           "loadgen.cpp", "http.cpp")]
    srcs.append(os.path.join(ROOT, "tests", "tsan", "fake_engine.cpp"))
    subprocess.run(["g++", "-std=c++17", "-O2", "-march=native", "-fPIC", "-shared", "-pthread",
                    *srcs, "-o", so], check=True)
    L = ctypes.CDLL(so)
    vp, cp = ctypes.c_void_p, ctypes.c_char_p
    L.vs_open.argtypes = [vp, ctypes.POINTER(vp)]
    L.vs_close.argtypes = [vp]
    L.vsvc_open.argtypes = [vp, cp, ctypes.POINTER(vp)]
    L.vsvc_close.argtypes = [vp]
    L.vsvc_http_start.argtypes = [vp, cp, ctypes.POINTER(vp)]
    L.vsvc_http_port.argtypes = [vp]
    L.vsvc_http_stop.argtypes = [vp]
    L.vsvc_loadgen.argtypes = [vp, cp, ctypes.POINTER(vp)]
    L.vsvc_free.argtypes = [vp]
    eng, svc, h = vp(), vp(), vp()
    assert L.vs_open(None, ctypes.byref(eng)) == 0
    assert L.vsvc_open(eng, None, ctypes.byref(svc)) == 0
    assert L.vsvc_http_start(svc, b"127.0.0.1:0", ctypes.byref(h)) == 0
    port = L.vsvc_http_port(h)
    try:
        _ingest(port, np.random.default_rng(7))

        def lg(spec):
            out = vp()
            assert L.vsvc_loadgen(None, json.dumps(spec).encode(), ctypes.byref(out)) == 0
            rep = json.loads(ctypes.string_at(out.value))
            L.vsvc_free(out)
            return rep
        return _measure(lg, port, "cpu (exact brute-force scan, test double)", seconds)
    finally:
        L.vsvc_http_stop(h)
        L.vsvc_close(svc)
        L.vs_close(eng)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", default="both", choices=["gpu", "cpu", "both"])
    ap.add_argument("--seconds", type=float, default=3.0)
    args = ap.parse_args()
    if args.backend in ("cpu", "both"):
        run_cpu(args.seconds)
    if args.backend in ("gpu", "both"):
        run_gpu(args.seconds)


if __name__ == "__main__":
    main()
