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
import resource
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)



def _cpu_quota():
    """CPUs the cgroup grants (cpu.max), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()
        return None if q == "max" else round(int(q) / int(p), 2)
    except Exception:
        return None

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
    ap.add_argument("--server", action="store_true",
                    help="serve from a separate lib/vsearch_server process (HTTP only)")
    ap.add_argument("--devices", default="0", help="--server: VS_DEVICES of the server")
    ap.add_argument("--placement", default="stripes", choices=["stripes", "collections"],
                    help="--server: VS_PLACEMENT of the server (with several devices)")
    ap.add_argument("--workers-default", action="store_true",
                    help="--server: leave the batcher's worker count to the service "
                         "(two per device the collections use)")
    args = ap.parse_args()
    if args.server:
        return run_server(args)
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
            ru0, w0 = resource.getrusage(resource.RUSAGE_SELF), time.time()
            rep = svc.loadgen(names, args.dim, clients=clients, seconds=args.seconds,
                              seed=clients, http=addr)
            ru1, w1 = resource.getrusage(resource.RUSAGE_SELF), time.time()
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
                    "largest_call": st["largest_call"],
                    # (r05) host CPU the process used over the run (clients,
                    # listener, batcher, engine host side), in CPUs busy
                    "host_cpus_busy": round((ru1.ru_utime - ru0.ru_utime + ru1.ru_stime - ru0.ru_stime)
                                            / max(w1 - w0, 1e-9), 2),
                    "cpu_quota": _cpu_quota()}
            print(json.dumps(line), flush=True)
        if lis is not None:
            lis.stop()
        svc.close()
        eng.close()


def run_server(args):
    """C5 against the vector-service process: lib/vsearch_server holds the
    three collections (VS_BULK) and serves them on a port; this process only
    drives retrieval-service-shaped HTTP load at it (vsvc_loadgen's client,
    no engine here)."""
    import ctypes
    import json as js
    import signal
    import subprocess
    import tempfile
    import __graft_entry__ as ge
    from importlib import import_module
    pkg = ge.load_package()
    svcmod = import_module(pkg.__name__ + ".service")
    L = svcmod.load_service_library()
    names = ["regulatory_docs", "merchant_docs", "kyc_docs"]
    batching = {"lead_us": args.lead_us}
    if not args.workers_default:
        batching["workers"] = args.workers
    cfg = {"collections": [{"name": n, "dim": args.dim, "metric": "Cosine", "dtype": "bf16"}
                           for n in names],
           "batching": batching}
    d = tempfile.mkdtemp(prefix="c5srv")
    cfgp = os.path.join(d, "cfg.json")
    open(cfgp, "w").write(js.dumps(cfg))
    env = dict(os.environ, PORT="0", VS_SERVICE_CONFIG=cfgp, VS_DEVICES=args.devices,
               VS_PLACEMENT=args.placement,
               VS_BULK=",".join(f"{n}={args.rows}:{0x5EED + i}" for i, n in enumerate(names)))
    server = os.path.join(os.path.dirname(svcmod.SVC_LIB_PATH), "vsearch_server")
    t0 = time.time()
    p = subprocess.Popen([server], env=env, stdout=subprocess.PIPE, text=True)
    port = None
    for _ in range(50):
        line = p.stdout.readline()
        if "starting on port" in line:
            port = int(line.split()[-1])
            break
        if not line:
            break
    if port is None:
        p.kill()
        raise SystemExit("vsearch_server did not start")
    print(f"[c5] vsearch_server on port {port}, {len(names)} x {args.rows} x {args.dim} bf16 "
          f"in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    try:
        for clients in [int(c) for c in args.clients.split(",")]:
            for secs, seed in ((0.5, 1), (args.seconds, clients)):
                spec = {"collections": names, "dim": args.dim, "clients": clients,
                        "seconds": secs, "k_min": 3, "k_max": 50, "seed": seed,
                        "http": f"127.0.0.1:{port}"}
                out = ctypes.c_void_p()
                rc = L.vsvc_loadgen(None, js.dumps(spec).encode(), ctypes.byref(out))
                if rc != 0:
                    raise SystemExit(f"loadgen failed: {rc}")
                rep = js.loads(ctypes.string_at(out.value))
                L.vsvc_free(out)
            line = {"workload": f"C5: 3 x {args.rows} x {args.dim} bf16, k in [3,50], closed "
                                "loop, HTTP clients -> vsearch_server process",
                    "transport": "http (separate server process)", "clients": clients,
                    "devices": args.devices, "placement": args.placement,
                    "workers": "service default" if args.workers_default else args.workers,
                    "lead_us": args.lead_us,
                    "qps": round(rep["qps"], 1), "requests": rep["requests"],
                    "errors": rep["errors"], "first_error": rep["first_error"][:200],
                    "lat_ms": {k: round(v, 3) for k, v in rep["lat_ms"].items()}}
            print(js.dumps(line), flush=True)
    finally:
        p.send_signal(signal.SIGTERM)
        p.wait(timeout=120)


if __name__ == "__main__":
    main()
