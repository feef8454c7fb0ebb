#!/usr/bin/env python3
"""Overlap of two concurrent host calls on a sharded engine, measured in
interleaved trials (moved out of the -x GPU suite).

A vs_open_multi engine holds the devices' work locks only while a call
enqueues (pinned per-call staging, the wait outside the locks), so two
threads should finish a pair of calls in well under twice one call's time.
Each trial times `calls` single-thread calls, then `calls` calls on each of
two threads, alternating; the record holds every trial's ratio, their median
and the fraction of trials under the stated 1.6 bound.

    python tools/concurrency_overlap.py [--trials 9] [--calls 300] [--out FILE]
"""
import argparse
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--trials", type=int, default=9)
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--bound", type=float, default=1.6)
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import __graft_entry__ as ge
    from oracle import oracle as orc
    pkg = ge.load_package()
    eng = pkg.VectorEngine(shards=[0, 0, 0, 0])
    dim, n = 256, 20_000
    eng.create_collection("ov", dim, 1, 1, n)
    eng.generate("ov", n, orc.SEED_CORPUS)
    Q = orc.generate(orc.SEED_QUERY, 3, 2, dim)
    want = [eng.search("ov", Q[i:i + 1], 10) for i in range(2)]
    bad = [0]

    def run(i):
        for _ in range(a.calls):
            s, r, c = eng.search("ov", Q[i:i + 1], 10)
            bad[0] += not np.array_equal(r, want[i][1])

    for _ in range(50):
        eng.search("ov", Q[:1], 10)
    ratios, ones, twos = [], [], []
    for t in range(a.trials):
        t0 = time.perf_counter()
        run(0)
        one = time.perf_counter() - t0
        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        t0 = time.perf_counter()
        for x in th:
            x.start()
        for x in th:
            x.join()
        two = time.perf_counter() - t0
        ones.append(one * 1e6 / a.calls)
        twos.append(two * 1e6 / a.calls)
        ratios.append(two / one)
        print(f"trial {t}: one {ones[-1]:.1f} us/call, pair {twos[-1]:.1f} us, ratio {ratios[-1]:.2f}",
              flush=True)
    eng.close()
    rec = {"tool": "tools/concurrency_overlap.py", "engine": "vs_open_multi shards [0,0,0,0]",
           "collection": f"{n} x {dim} bf16 dot", "calls_per_trial": a.calls,
           "trials": a.trials, "one_thread_us_per_call": [round(x, 2) for x in ones],
           "two_threads_us_per_pair": [round(x, 2) for x in twos],
           "ratio": [round(x, 3) for x in ratios], "ratio_median": round(statistics.median(ratios), 3),
           "bound": a.bound, "trials_under_bound": sum(r < a.bound for r in ratios),
           "wrong_answers": bad[0], "build_id": pkg.build_id()}
    print(json.dumps(rec))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rec, f, indent=1)
    return 0 if bad[0] == 0 else 1


if __name__ == "__main__":
    sys.exit(main())
