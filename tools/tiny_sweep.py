"""Single-query latency of small fp32 collections through the host API
(vs_search: staging copy, query prep, GEMV scan, merge, copy back), for the
GEMV grid's rows-per-wave floor (VS_GEMV_MIN_RPW, read once per process).

    VS_GEMV_MIN_RPW=4 python tools/tiny_sweep.py
    VS_SWEEP_ROWS=2000,200000 VS_SWEEP_K=10,100 VS_SWEEP_DTYPE=bf16 python tools/tiny_sweep.py

One JSON line: p50 / p10 latency in microseconds per (rows, k). VS_SWEEP_*
pick the sizes, k values and dtype (default 221..200k rows, k 5 / 100, fp32);
VS_LARGE_K_FROM (read once by the library) moves the list / large-k split.
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401  (binds torch's HIP runtime first, as bench.py does)
    import __graft_entry__ as ge
    pkg = ge.load_package()
    eng = pkg.VectorEngine(device=0)
    rows_l = [int(x) for x in os.environ.get("VS_SWEEP_ROWS", "221,2000,20000,200000").split(",")]
    ks = [int(x) for x in os.environ.get("VS_SWEEP_K", "5,100").split(",")]
    dt = os.environ.get("VS_SWEEP_DTYPE", "f32")
    out = {"min_rpw": os.environ.get("VS_GEMV_MIN_RPW", "2 (default)"),
           "large_k_from": os.environ.get("VS_LARGE_K_FROM", "129 (default)"), "dtype": dt,
           "lat_us": {}}
    rng = np.random.default_rng(1)
    try:
        for rows in rows_l:
            name = f"t{rows}"
            eng.create_collection(name, 768, pkg.METRIC_COSINE,
                                  pkg.DTYPE_BF16 if dt == "bf16" else pkg.DTYPE_F32)
            eng.generate(name, rows, 5)
            q = rng.standard_normal((1, 768)).astype(np.float32)
            for k in ks:
                for _ in range(200):
                    eng.search(name, q, k)
                ts = []
                for _ in range(2000):
                    t0 = time.perf_counter()
                    eng.search(name, q, k)
                    ts.append(time.perf_counter() - t0)
                ts = np.array(ts) * 1e6
                out["lat_us"][f"{rows}/k{k}"] = [round(float(np.percentile(ts, 50)), 1),
                                                 round(float(np.percentile(ts, 10)), 1)]
            eng.drop_collection(name)
    finally:
        eng.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
