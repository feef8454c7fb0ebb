#!/usr/bin/env python3
"""r06: where the N = 8 share's bench step spends what share_pipe does not
see. 1.25M x 768 bf16, 256 fresh queries a step, k = 10 (the share), timed
three ways on one engine: vs_search_keys straight from Python, the bench's
ShardedSearch wrapper, and the wrapper with the engine's sampled timing.
Per arm: host enqueue time per step (before the synchronize) and wall time
per step. One JSON line."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import __graft_entry__ as ge  # noqa: E402


def main():
    pkg = ge.load_package()
    from importlib import import_module
    shard = import_module(pkg.__name__ + ".shard")
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 1_250_000
    dim, k, nq, steps = 768, 10, 256, 200
    res = {}
    for name, kw in (("plain", dict()), ("timing_sampled", dict(timing=True, timing_sample=True))):
        e = pkg.VectorEngine(device=0, **kw)
        e.create_collection("s", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, rows, 0)
        e.generate("s", rows, 0x5EED)
        stream_fn = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
        nb = 2 * (steps + 20)
        q = torch.empty((nb, nq, dim), dtype=torch.float32, device="cuda")
        e.generate_vectors(0xC0FFEE, 0, nb * nq, dim, q.data_ptr(), stream_fn())
        outs = [torch.empty((nq, k), dtype=torch.int64, device="cuda") for _ in range(steps)]
        ls, mg = shard.engine_callables(e, "s", dim, stream_fn, reuse=True, ring=steps)
        sh = shard.ShardedSearch(ls, mg)
        arms = {"direct": lambda i, j: e.search_keys("s", q[i].data_ptr(), nq, dim, k,
                                                     outs[j].data_ptr(), stream_fn()),
                "sharded": lambda i, j: sh.search(q[i], k)}
        base = 0
        for rep in range(2):
            for an, f in arms.items():
                for i in range(20):
                    f(base + i, i)
                base += 20
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for j in range(steps):
                    f(base + j, j)
                t1 = time.perf_counter()
                torch.cuda.synchronize()
                t2 = time.perf_counter()
                base = (base + steps) % (nb - steps - 20)
                key = f"{name}_{an}"
                res.setdefault(key, []).append({"host_us": round((t1 - t0) / steps * 1e6, 2),
                                                "step_us": round((t2 - t0) / steps * 1e6, 2)})
                print(key, res[key][-1], file=sys.stderr, flush=True)
        e.close() if hasattr(e, "close") else None
        del e
        torch.cuda.synchronize()
    print(json.dumps({"tool": "s125_host_probe", "rows": rows, "nq": nq, "k": k, "steps": steps,
                      "arms": res}))


if __name__ == "__main__":
    main()
