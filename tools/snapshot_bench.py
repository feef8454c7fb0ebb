"""Snapshot / restore / checksum throughput on one GPU.

    python tools/snapshot_bench.py [--rows 10000000] [--snap-rows 1000000] [--dir /tmp]

checksum: the device reduction over the whole collection (HBM-bound; bytes =
rows x dim x 2), timed over repeated calls. snapshot / restore: file write and
read through pinned staging, timed end to end on a smaller collection (the
file lands in --dir and is deleted afterwards). One JSON line.
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
    ap.add_argument("--snap-rows", type=int, default=1_000_000)
    ap.add_argument("--dim", type=int, default=768)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--dir", default="/tmp")
    args = ap.parse_args()
    import torch  # noqa: F401
    import __graft_entry__ as ge
    pkg = ge.load_package()
    eng = pkg.VectorEngine(device=0)
    eng.create_collection("big", args.dim, 1, 1, args.rows)
    eng.generate("big", args.rows, 0x5EED)
    eng.checksum("big")
    t0 = time.perf_counter()
    for _ in range(args.reps):
        h = eng.checksum("big")
    dt = (time.perf_counter() - t0) / args.reps
    nbytes = args.rows * args.dim * 2
    out = {"checksum": {"rows": args.rows, "bytes": nbytes, "ms": round(dt * 1e3, 3),
                        "GBps": round(nbytes / dt / 1e9, 1), "value": hex(h)}}
    eng.drop_collection("big")
    eng.create_collection("s", args.dim, 1, 1, args.snap_rows)
    eng.generate("s", args.snap_rows, 0x5EED)
    path = os.path.join(args.dir, f"vsnap_bench_{os.getpid()}.vsnap")
    try:
        t0 = time.perf_counter()
        eng.snapshot("s", path)
        ts = time.perf_counter() - t0
        t0 = time.perf_counter()
        eng.restore("r", path)
        tr = time.perf_counter() - t0
        sb = args.snap_rows * args.dim * 2
        assert eng.checksum("r") == eng.checksum("s")
        out["snapshot"] = {"rows": args.snap_rows, "bytes": sb, "s": round(ts, 3),
                           "GBps": round(sb / ts / 1e9, 2)}
        out["restore"] = {"rows": args.snap_rows, "bytes": sb, "s": round(tr, 3),
                          "GBps": round(sb / tr / 1e9, 2)}
    finally:
        if os.path.exists(path):
            os.remove(path)
    print(json.dumps(out), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
