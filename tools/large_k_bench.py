"""Single-query search time against k, across the list path (k <= 1024) and
the large-k path (score pass + device radix select + sort, vs_select.hip).

    python tools/large_k_bench.py [--rows 10000000] [--dim 768] [--dtype bf16] [--reps 20]

One JSON line per k: median / min wall time of vs_search (host API, one
query, results decoded on the host) and the scan kernel's HIP-event time
(VS_FLAG_TIMING: the score pass on the large-k path, the GEMV scan on the
list path), with the scan's HBM rate. Run under rocprofv3 --kernel-trace
--stats for the per-kernel split (score pass, hist / pick / compact, sort).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=10_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "f32"])
    ap.add_argument("--ks", default="10,1024,1025,2000,5000,50000,500000")
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import torch  # noqa: F401  (binds torch's HIP runtime first, as bench.py does)
    import __graft_entry__ as ge
    from oracle import oracle as orc
    pkg = ge.load_package()
    bf16 = args.dtype == "bf16"
    eng = pkg.VectorEngine(device=0, timing=True)
    eng.create_collection("lk", args.dim, pkg.METRIC_DOT, pkg.DTYPE_BF16 if bf16 else pkg.DTYPE_F32,
                          args.rows)
    eng.generate("lk", args.rows, orc.SEED_CORPUS)
    Q = orc.generate(orc.SEED_QUERY, 0, args.reps + 3, args.dim)
    row_bytes = args.dim * (2 if bf16 else 4)
    for k in [int(x) for x in args.ks.split(",")]:
        for i in range(3):
            eng.search("lk", Q[i], k)
        eng.timing(reset=True)
        ts = []
        for i in range(args.reps):
            t0 = time.perf_counter()
            s, r, c = eng.search("lk", Q[3 + i], k)
            ts.append(time.perf_counter() - t0)
        tm = eng.timing(reset=True)
        assert int(c[0]) == min(k, args.rows) and np.all(np.diff(s[0, :int(c[0])]) <= 0)
        scan_ms = tm["scan_ms"]
        print(json.dumps({
            "workload": f"{args.rows} x {args.dim} {args.dtype}, one query, inner product",
            "k": k, "path": "large-k (score pass + radix select + sort)" if k > 1024 else "list",
            "wall_ms_median": round(float(np.median(ts)) * 1e3, 4),
            "wall_ms_min": round(float(np.min(ts)) * 1e3, 4),
            "scan_ms": round(scan_ms, 4),
            "scan_hbm_gbs": round(args.rows * row_bytes / (scan_ms / 1e3) / 1e9, 1) if scan_ms else None,
            "reps": args.reps}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
