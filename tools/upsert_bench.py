#!/usr/bin/env python3
"""Store-side throughput: vs_upsert into HBM and the
/upsert handler mirror with ingest-service's bodies.

    python tools/upsert_bench.py [--rows 1000000] [--dim 768] [--parts engine,service]
                                 [--out FILE]
    (VS_UPSERT_CHUNK_MB=N sets the engine's staging chunk, default 16)

Engine: a Cosine collection is filled by appends of `batch` rows from host
fp32 arrays (the vectors are normalised on the device, as Qdrant's
cosine_preprocess does at upsert), then `batch` existing rows are
overwritten in shuffled order; per call: wall time, input GB/s (fp32 bytes
from the host), rows/s. fp32 and bf16 collections.
Service: bodies shaped like rag/ingest-service/main.go:359-386 (storeVectors:
one /upsert per document, here 110 chunks of ~500-rune text, 768 numbers per
vector) through vsvc_handle, from 1 and 8 threads: points/s and MB/s of JSON.
Every call's answer is checked (rows stored = read back; HTTP 200 bodies).
"""
import argparse
import json
import os
import sys
import threading
import time
import uuid

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def engine_part(pkg, rows, dim, batches, dtype):
    out = []
    eng = pkg.VectorEngine(device=0)
    rng = np.random.default_rng(5)
    X = rng.standard_normal((rows, dim), dtype=np.float32)
    try:
        for b in batches:
            name = f"up_{dtype}_{b}"
            eng.create_collection(name, dim, pkg.METRIC_COSINE, dtype, rows)
            eng.upsert(name, np.arange(min(b, rows)), X[:min(b, rows)])  # warm (allocs, page-in)
            times = []
            t_all = time.perf_counter()
            for o in range(min(b, rows), rows, b):
                n = min(b, rows - o)
                t0 = time.perf_counter()
                eng.upsert(name, np.arange(o, o + n, dtype=np.uint64), X[o:o + n])
                times.append((n, time.perf_counter() - t0))
            el = time.perf_counter() - t_all
            got = eng.read_rows(name, rows - 3, 3)
            want = X[rows - 3:] / np.linalg.norm(X[rows - 3:], axis=1, keepdims=True)
            tol = 1e-2 if dtype == pkg.DTYPE_BF16 else 1e-6
            assert np.allclose(got, want, atol=tol), "stored rows differ"
            n_app = sum(n for n, _ in times)
            med = sorted(t / n for n, t in times)[len(times) // 2] if times else 0
            ids = rng.permutation(rows)[:b].astype(np.uint64)
            t0 = time.perf_counter()
            eng.upsert(name, ids, X[:len(ids)])
            ow = time.perf_counter() - t0
            rec = {"part": "engine vs_upsert", "dtype": "bf16" if dtype else "f32", "dim": dim,
                   "batch_rows": b, "appended_rows": n_app,
                   "append_rows_per_s": round(n_app / el), "append_input_gbs": round(n_app * dim * 4 / el / 1e9, 2),
                   "append_median_us_per_row": round(med * 1e6, 3),
                   "overwrite_rows": len(ids), "overwrite_s": round(ow, 4),
                   "overwrite_rows_per_s": round(len(ids) / ow)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
            eng.drop_collection(name)
    finally:
        eng.close()
    return out


WORDS = ["RBI", "shall", "merchant", "KYC", "payment", "aggregator", "settlement", "escrow",
         "account", "compliance", "directions", "regulated", "entity", "customer"]


def bodies(n_docs, chunks, dim, seed=7):
    rng = np.random.default_rng(seed)
    out = []
    for d in range(n_docs):
        pts = []
        for i in range(chunks):
            v = rng.standard_normal(dim)
            pts.append({"id": str(uuid.UUID(bytes=rng.bytes(16), version=4)),
                        "vector": [float(x) for x in v.astype(np.float32)],
                        "payload": {"text": " ".join(rng.choice(WORDS, 80))[:500],
                                    "document_id": f"doc-{seed}-{d}", "position": i}})
        out.append(json.dumps({"collection": "regulatory_docs", "points": pts}).encode())
    return out


def service_part(pkg, svcmod, dim, n_docs, chunks):
    out = []
    for threads in (1, 8):
        eng = pkg.VectorEngine(device=0)
        svc = svcmod.VectorService(eng)  # the reference's 3 x 768 Cosine collections
        try:
            bs = bodies(n_docs, chunks, dim, seed=threads)
            svc.handle("POST", "/upsert", bodies(1, chunks, dim, seed=99)[0])  # warm
            mb = sum(len(b) for b in bs) / 1e6
            bad = []
            per = [bs[i::threads] for i in range(threads)]

            def run(mine):
                for b in mine:
                    st, body, _ = svc.handle("POST", "/upsert", b)
                    if st != 200:
                        bad.append((st, body[:200]))

            th = [threading.Thread(target=run, args=(p,)) for p in per]
            t0 = time.perf_counter()
            for t in th:
                t.start()
            for t in th:
                t.join()
            el = time.perf_counter() - t0
            assert not bad, bad[:2]
            rows = eng.collection_info("regulatory_docs")["rows"]
            assert rows == n_docs * chunks + chunks, rows
            rec = {"part": "service /upsert (vsvc_handle)", "threads": threads, "docs": n_docs,
                   "points_per_body": chunks, "points": n_docs * chunks,
                   "points_per_s": round(n_docs * chunks / el), "json_mb_per_s": round(mb / el, 1),
                   "ms_per_body": round(el / n_docs * 1e3, 3)}
            print(json.dumps(rec), flush=True)
            out.append(rec)
        finally:
            svc.close()
            eng.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--docs", type=int, default=200)
    ap.add_argument("--out", default="")
    ap.add_argument("--parts", default="engine,service")
    a = ap.parse_args()
    import __graft_entry__ as ge
    from importlib import import_module
    pkg = ge.load_package()
    svcmod = import_module(pkg.__name__ + ".service")
    recs = []
    if "engine" in a.parts:
        for dtype in (pkg.DTYPE_F32, pkg.DTYPE_BF16):
            recs += engine_part(pkg, a.rows, a.dim, (10_000, 100_000), dtype)
    if "service" in a.parts:
        recs += service_part(pkg, svcmod, a.dim, a.docs, 110)
    for r in recs:
        r["chunk_mb"] = os.environ.get("VS_UPSERT_CHUNK_MB", "16")
    if a.out:
        with open(a.out, "w") as f:
            for r in recs:
                f.write(json.dumps(r) + "\n")


if __name__ == "__main__":
    main()
