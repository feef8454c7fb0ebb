"""Filtered single-query search cost vs filter density.

    python tools/filter_bench.py [--rows 10000000] [--dim 768] [--reps 50]

For each density the same random bitmap is used for --reps single-query
vs_search_filtered calls (host bitmap in, host results out). Reported: wall
ms per call, the scan kernel's HIP-event ms, and for the gather path (density
<= 1/8) the gathered row bytes / kernel time. One JSON line.
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
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--k", type=int, default=10)
    args = ap.parse_args()
    import torch  # noqa: F401
    import __graft_entry__ as ge
    pkg = ge.load_package()
    from oracle import oracle as orc  # query generator only (same seeds as bench.py)
    eng = pkg.VectorEngine(device=0, timing=True)
    eng.create_collection("big", args.dim, 1, 1, args.rows)
    eng.generate("big", args.rows, orc.SEED_CORPUS)
    Q = orc.generate(orc.SEED_QUERY, 0, args.reps, args.dim)
    rng = np.random.default_rng(1)
    out = {"workload": f"{args.rows} x {args.dim} bf16, single query, top-{args.k}",
           "densities": []}
    for dens in (1.0, 0.5, 0.125, 0.05, 0.01, 0.001):
        mask = pkg.pack_allow(rng.random(args.rows) < dens)
        for i in range(3):
            eng.search_filtered("big", Q[i], args.k, mask)
        eng.timing(reset=True)
        t0 = time.perf_counter()
        for i in range(args.reps):
            eng.search_filtered("big", Q[i], args.k, mask)
        wall = (time.perf_counter() - t0) / args.reps
        tm = eng.timing(reset=True)
        scan = tm["scan_ms"]  # vs_timing reports the average per scan
        allowed = int(np.unpackbits(mask.view(np.uint8)).sum())
        row = {"density": dens, "allowed": allowed, "wall_ms": round(wall * 1e3, 4),
               "scan_ms": round(scan, 4), "qps": round(1.0 / wall, 1)}
        if allowed * 8 <= args.rows:
            row["gather_gbs"] = round(allowed * args.dim * 2 / (scan * 1e-3) / 1e9, 1)
        else:
            row["stream_gbs"] = round(args.rows * args.dim * 2 / (scan * 1e-3) / 1e9, 1)
        out["densities"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    # the same single-query searches through a device-resident filter
    # (vs_filter_create once, then vs_search_filter_id: no bitmap per call)
    out["resident"] = []
    for dens in (0.125, 0.01, 0.001):
        fid = eng.filter_create("big", rng.random(args.rows) < dens)
        for i in range(3):
            eng.search_filter_id("big", Q[i], args.k, fid)
        eng.timing(reset=True)
        t0 = time.perf_counter()
        for i in range(args.reps):
            eng.search_filter_id("big", Q[i], args.k, fid)
        wall = (time.perf_counter() - t0) / args.reps
        tm = eng.timing(reset=True)
        eng.filter_drop(fid)
        row = {"density": dens, "wall_ms": round(wall * 1e3, 4),
               "scan_ms": round(tm["scan_ms"], 4), "qps": round(1.0 / wall, 1)}
        out["resident"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    # fixed cost of one host-API search (tiny collection, no filter)
    eng.create_collection("tiny", args.dim, 1, 1, 1000)
    eng.generate("tiny", 1000, orc.SEED_CORPUS)
    for i in range(3):
        eng.search("tiny", Q[i], args.k)
    t0 = time.perf_counter()
    for i in range(args.reps):
        eng.search("tiny", Q[i], args.k)
    out["tiny_unfiltered_wall_ms"] = round((time.perf_counter() - t0) / args.reps * 1e3, 4)
    print(json.dumps({"tiny_unfiltered_wall_ms": out["tiny_unfiltered_wall_ms"]}), file=sys.stderr)
    # batches of 8 queries: the MFMA pass with the bitmap fused (dense
    # filters) or 8 gathered scans (selective filters, search_core's rule)
    out["batch8"] = []
    for dens in (0.5, 0.05, 0.01, 0.001):
        mask = pkg.pack_allow(rng.random(args.rows) < dens)
        for i in range(3):
            eng.search_filtered("big", Q[:8], args.k, mask)
        t0 = time.perf_counter()
        for i in range(args.reps // 5):
            eng.search_filtered("big", Q[:8], args.k, mask)
        wall = (time.perf_counter() - t0) / (args.reps // 5)
        row = {"density": dens, "nq": 8, "wall_ms": round(wall * 1e3, 4),
               "qps": round(8 / wall, 1)}
        out["batch8"].append(row)
        print(json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out))
    eng.close()


if __name__ == "__main__":
    main()
