"""Config C5 (BASELINE.json): closed-loop concurrent /search traffic through the
vector-service mirror, 3 collections x 5M x 1024 bf16, k uniform in [3, 50].

    python tools/loadgen_c5.py [--rows 5000000] [--clients 16,64,256] [--seconds 5]
                               [--transport inproc|http|both]

Each client count runs once with the dynamic batcher (csrc/service/batcher.h)
and, for comparison, once with batching off. Clients are threads sending
retrieval-service-shaped JSON bodies (csrc/service/loadgen.cpp): in-process
through vsvc_handle, or (--transport http) as HTTP/1.1 POSTs over TCP to the
service's listener (vsvc_http_start on 127.0.0.1), each client on its own
keep-alive connection. One JSON line per run.
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
    ap.add_argument("--rows", type=int, default=5_000_000)
    ap.add_argument("--dim", type=int, default=1024)
    ap.add_argument("--clients", default="16,64,256")
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--unbatched-clients", type=int, default=64)
    ap.add_argument("--workers", type=int, default=2, help="batcher worker threads")
    ap.add_argument("--lead-us", type=int, default=300,
                    help="late batch formation with a call in flight (batcher.h)")
    ap.add_argument("--transport", default="inproc", choices=["inproc", "http", "both"])
    args = ap.parse_args()
    import torch  # noqa: F401  (binds torch's HIP runtime first, as bench.py does)
    import __graft_entry__ as ge
    from importlib import import_module
    pkg = ge.load_package()
    svcmod = import_module(pkg.__name__ + ".service")
    names = ["regulatory_docs", "merchant_docs", "kyc_docs"]
    colls = [{"name": n, "dim": args.dim, "metric": "Cosine", "dtype": "bf16"} for n in names]
    runs = [(int(c), True) for c in args.clients.split(",")]
    if args.unbatched_clients:
        runs.append((args.unbatched_clients, False))
    for batching in (True, False):
        todo = [c for c, b in runs if b == batching]
        if not todo:
            continue
        eng = pkg.VectorEngine(device=0)
        svc = svcmod.VectorService(eng, {"collections": colls,
                                         "batching": {"enabled": batching,
                                                      "workers": args.workers,
                                                      "lead_us": args.lead_us}})
        t0 = time.time()
        for i, n in enumerate(names):
            svc.bulk_generate(n, args.rows, 0x5EED + i)
        print(f"[c5] {len(names)} x {args.rows} x {args.dim} bf16 generated in "
              f"{time.time() - t0:.1f}s", file=sys.stderr, flush=True)
        lis = svc.serve("127.0.0.1:0") if args.transport != "inproc" else None
        transports = ["inproc", "http"] if args.transport == "both" else [args.transport]
        for clients, transport in [(c, t) for c in todo for t in transports]:
            addr = "127.0.0.1:%d" % lis.port if transport == "http" else None
            svc.loadgen(names, args.dim, clients=clients, seconds=0.5, http=addr)  # warm-up
            before = svc.stats()
            rep = svc.loadgen(names, args.dim, clients=clients, seconds=args.seconds,
                              seed=clients, http=addr)
            st = svc.stats()
            calls = st["engine_calls"] - before["engine_calls"]
            nreq = st["requests"] - before["requests"]
            line = {"workload": f"C5: 3 x {args.rows} x {args.dim} bf16, k in [3,50], "
                                f"closed loop, {transport} clients",
                    "transport": transport, "clients": clients, "batching": batching, "workers": args.workers, "lead_us": args.lead_us,
                    "qps": round(rep["qps"], 1),
                    "requests": rep["requests"], "errors": rep["errors"],
                    "first_error": rep["first_error"][:200],
                    "lat_ms": {k: round(v, 3) for k, v in rep["lat_ms"].items()},
                    "engine_calls": calls,
                    "mean_batch": round(nreq / calls, 2) if calls else None,
                    "largest_call": st["largest_call"]}
            print(json.dumps(line), flush=True)
        if lis is not None:
            lis.stop()
        svc.close()
        eng.close()


if __name__ == "__main__":
    main()
