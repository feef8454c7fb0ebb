#!/usr/bin/env python3
"""r06: does the engine's sampled event timing cost the C2 line anything?
C2's workload (1M x 768 fp32, cosine, one query, k = 10) searched by an
engine with timing=True, timing_sample=True (bench.py's) and one with timing
off, fresh queries per step, arms interleaved. One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    rows, dim, k, steps = 1_000_000, 768, 10, 400
    stream = torch.cuda.current_stream().cuda_stream
    arms = {}
    for name, kw in (("timing_sampled", dict(timing=True, timing_sample=True)),
                     ("timing_off", dict())):
        e = pkg.VectorEngine(device=0, **kw)
        e.create_collection("c2", dim, pkg.METRIC_COSINE, pkg.DTYPE_F32, rows, 0)
        e.generate("c2", rows, 0x5EED)
        arms[name] = e
    q = torch.empty((steps + 10, dim), dtype=torch.float32, device="cuda")
    arms["timing_off"].generate_vectors(0xC0FFEE, 0, steps + 10, dim, q.data_ptr(), stream)
    outs = [torch.empty((1, k), dtype=torch.int64, device="cuda") for _ in range(steps + 10)]
    res = {n: [] for n in arms}
    for rep in range(3):
        for n, e in arms.items():
            for i in range(10):
                e.search_keys("c2", q[i].data_ptr(), 1, dim, k, outs[i].data_ptr(), stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(10, steps + 10):
                e.search_keys("c2", q[i].data_ptr(), 1, dim, k, outs[i].data_ptr(), stream)
            torch.cuda.synchronize()
            res[n].append(round((time.perf_counter() - t0) / steps * 1e6, 2))
            print(n, res[n][-1], flush=True, file=sys.stderr)
    print(json.dumps({"tool": "c2_timing_ab", "rows": rows, "k": k, "steps": steps,
                      "us_per_query": res,
                      "qps_median": {n: round(1e6 / sorted(v)[1], 1) for n, v in res.items()}}))


if __name__ == "__main__":
    main()
