#!/usr/bin/env python3
"""Timing arms of the int8 prefilter pass (r04): one process per arm, since
VS_Q8_VAR (the pass's compile-time variant) is read once.

    VS_Q8_VAR=2304 python tools/q8_arms.py [--rows 10000000] [--steps 30] [--k 10]
    VS_Q8_SAMPLE=2 python tools/q8_arms.py ...   (sample tiles x2)

Prints one JSON line: the arm, the int8 pass's average HIP-event duration
(every launch bracketed), ms per step and QPS. No answer is checked (the
no-append arm returns wrong ones by design); the product arm's answers are
checked by bench.py and the GPU tests.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--k", type=int, default=10)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--cosine", action="store_true")
    a = ap.parse_args()
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    eng = pkg.VectorEngine(device=0, timing=True)
    eng.create_collection("b", a.dim, pkg.METRIC_COSINE if a.cosine else pkg.METRIC_DOT,
                          pkg.DTYPE_BF16, a.rows)
    eng.generate("b", a.rows, 0x5EED)
    q = torch.empty((256, a.dim), dtype=torch.float32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    eng.generate_vectors(0xC0FFEE, 0, 256, a.dim, q.data_ptr(), st)
    keys = torch.empty((256, a.k), dtype=torch.int64, device="cuda")
    for _ in range(a.warmup):
        eng.search_keys("b", q.data_ptr(), 256, a.dim, a.k, keys.data_ptr(), st)
    torch.cuda.synchronize()
    eng.timing(reset=True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        eng.search_keys("b", q.data_ptr(), 256, a.dim, a.k, keys.data_ptr(), st)
    torch.cuda.synchronize()
    el = time.perf_counter() - t0
    tm = eng.timing(reset=True)
    print(json.dumps({"arm": os.environ.get("VS_Q8_VAR", "default"),
                      "sample": os.environ.get("VS_Q8_SAMPLE", "1"), "k": a.k, "dim": a.dim, "rows": a.rows,
                      "prefilter_bytes": eng.prefilter_bytes("b"),
                      "scan_ms": round(tm["scan_ms"], 4), "scans": tm["scan_n"],
                      "ms_per_step": round(el / a.steps * 1e3, 4),
                      "qps": round(256 * a.steps / el, 1)}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
