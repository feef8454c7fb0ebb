#!/usr/bin/env python3
"""Benchmark of the exact top-k search engine (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c3|c3b1|c2]

A "step" is one pass of the hot path over one batch of queries: scan of the
whole (row-sharded) corpus, fused per-GPU top-k, RCCL all-gather of the local
lists (N > 1), on-device merge. Inputs (corpus and queries) are resident in
HBM before the timed region; nothing is skipped inside it.

Default workload (config c3 = BASELINE.json configs[2], the only config quoted
on a 10M x 768 corpus with top-10): 10,000,000 x 768 bf16 synthetic unit rows,
256-query batches, top-10, inner product. Scaling is strong: the corpus is
fixed and row-sharded over the N GPUs; value = queries/s of the whole job.

Prints ONE JSON line on rank 0 (driver contract), with "roofline" for the
dominant kernel (HIP-event durations on the engine's stream) and
"cpu_baseline" (oracle/ CPU scan timed on this host, rank 0, N = 1 only).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0            # MI355X HBM3E spec (MI355X_MICROARCH.md)
BF16_DENSE_TFLOPS = 2516.6       # 256 CU x 4096 flop/clk x 2.4 GHz (dense, no sparsity)
F32_MFMA_TFLOPS = 157.3          # v_mfma_f32_16x16x4_f32: 1/16 of bf16 (MI355X_MICROARCH.md)
I8_DENSE_TOPS = 2 * BF16_DENSE_TFLOPS  # v_mfma_i32_16x16x64_i8: 2x the bf16 rate per clock

CONFIGS = {
    # name: (rows, dim, dtype, metric, batch, k, description; {rows} = the corpus size)
    "c3": (10_000_000, 768, "bf16", "dot", 256, 10,
           "C3: {rows} x 768 bf16 corpus, 256-query batches, exact top-10, inner product"),
    "c3b1": (10_000_000, 768, "bf16", "dot", 1, 10,
             "{rows} x 768 bf16 corpus, single query, exact top-10, inner product (GEMV)"),
    "c2": (1_000_000, 768, "f32", "cosine", 1, 10,
           "C2: {rows} x 768 fp32 corpus, single query, exact top-10, cosine (GEMV)"),
    # the reference's collection type (fp32) batched: f32 MFMA pass
    "c2b256": (1_000_000, 768, "f32", "cosine", 256, 10,
               "C2 corpus batched: {rows} x 768 fp32, 256-query batches, exact top-10, cosine "
               "(f32 MFMA)"),
    # the metric sweep's fp32 arm (N = 10M, D = 768, bf16 and
    # fp32, B in {1, 256}): the reference's collection dtype at the C3 size
    "c3f32": (10_000_000, 768, "f32", "dot", 256, 10,
              "{rows} x 768 fp32 corpus, 256-query batches, exact top-10, inner product "
              "(f32 MFMA)"),
    "c3f32b1": (10_000_000, 768, "f32", "dot", 1, 10,
                "{rows} x 768 fp32 corpus, single query, exact top-10, inner product (GEMV)"),
    # one C5 collection's scan at a full batch (C5 itself is a service load:
    # tools/loadgen_c5.py); 1024-d rows: 128 queries per MFMA launch
    "c5b256": (5_000_000, 1024, "bf16", "cosine", 256, 50,
               "C5 collection: {rows} x 1024 bf16, 256-query batches, exact top-50, cosine"),
    # C4 is quoted on 8 GPUs (12.5M rows each); on fewer GPUs each holds more
    # (100M x 768 bf16 = 153.6 GB fits one MI355X's 288 GB)
    "c4": (100_000_000, 768, "bf16", "dot", 256, 100,
           "C4: {rows} x 768 bf16 corpus row-sharded, 256-query batches, exact top-100, IP"),
    "c4b1": (100_000_000, 768, "bf16", "dot", 1, 100,
             "C4: {rows} x 768 bf16 corpus row-sharded, single query, exact top-100, IP (GEMV)"),
}


def fmt_rows(n: int) -> str:
    """10_000_000 -> '10M', 1_250_000 -> '1.25M', 300_000 -> '300k'."""
    if n >= 1_000_000:
        return f"{n / 1e6:g}M"
    if n >= 1000:
        return f"{n / 1e3:g}k"
    return str(n)
METRIC_NAME = "exact top-10 QPS on 10M×768 corpus at 1/2/4/8 GPUs; % of HBM/MFMA peak"
# configs other than c3 report their own workload under the same metric name
# only as secondary measurements (the driver's headline run uses the default)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # defaults: 50 / 10 for batched configs; 400 / 50 for one-query configs,
    # whose ~0.15 ms steps would otherwise time 7 ms, inside the clock's ramp
    # (r06: C2 at 50 steps 6.36k QPS, at 400 7.0k on the same build)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--config", default="c3", choices=sorted(CONFIGS))
    ap.add_argument("--rows", type=int, default=0, help="override corpus rows (testing only)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=0,
                    help="CPU baseline corpus rows (0 = the full corpus)")
    ap.add_argument("--cpu-budget-s", type=float, default=12.0,
                    help="time budget of each CPU baseline leg (per-query scan, batched BLAS)")
    ap.add_argument("--dump-keys", default="",
                    help="rank 0 writes the last step's merged keys here (.npy; parity tests)")
    a = ap.parse_args()
    one = CONFIGS[a.config][4] == 1
    if a.steps is None:
        a.steps = 400 if one else 50
    if a.warmup is None:
        a.warmup = 50 if one else 10
    return a


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def kernel_roofline(cfg_rows_local, dim, elem, batch, k, t_ms, bound, queries_per_pass=256):
    """Algorithmic work of one scan launch / its measured duration.

    A launch covers at most `queries_per_pass` queries (fp32 at dim 768: 128),
    so a batch of `batch` queries takes ceil(batch / qpp) launches; the work
    of ONE launch is priced against one launch's average duration."""
    per_launch = min(batch, queries_per_pass)
    passes = -(-batch // per_launch)
    bytes_ = cfg_rows_local * dim * elem + per_launch * dim * elem + per_launch * k * 12
    flops = 2.0 * per_launch * cfg_rows_local * dim
    t = t_ms / 1e3
    gbs = bytes_ / t / 1e9
    tfs = flops / t / 1e12
    if bound == "mfma":
        peak = BF16_DENSE_TFLOPS if elem == 2 else F32_MFMA_TFLOPS
        return {"bound": "mfma", "achieved": round(tfs, 2), "peak": peak,
                "unit": "TFLOP/s", "frac": round(tfs / peak, 4), "launches_per_step": passes,
                "hbm_achieved_gbs": round(gbs, 1), "hbm_frac": round(gbs / HBM_PEAK_GBS, 4),
                "kernel_ms": round(t_ms, 4), "bytes_per_launch": int(bytes_),
                "flops_per_launch": int(flops)}
    return {"bound": "hbm", "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "kernel_ms": round(t_ms, 4),
            "bytes_per_launch": int(bytes_)}


def int8_roofline(rows_local, dim, batch, k, t_ms, queries_per_pass=256):
    """The int8 prefilter pass (DESIGN.md §5 "int8 prefilter"): it streams the
    int8 copy (D bytes per row) and does 2 B D int8 MACs per row; at B = 256
    its intensity (512 op/B) is under the i8 ridge (5033 TOP/s / 8 TB/s = 629),
    so HBM is the roof it is priced against, with the MFMA figures beside it.
    `bf16_equivalent_throughput_frac` is the exact search's delivered work
    (the bf16 pass's 2 B N D flops) per second over the bf16 dense peak: a
    bf16-EQUIVALENT throughput, not MFMA utilisation. The north_star's >= 50%
    of bf16 MFMA peak is measured on the bf16 pass itself (the `bf16_pass`
    line's roofline.frac), never by this field."""
    per_launch = min(batch, queries_per_pass)
    bytes_ = rows_local * dim + per_launch * dim + per_launch * k * 12
    ops = 2.0 * per_launch * rows_local * dim
    t = t_ms / 1e3
    gbs, tops = bytes_ / t / 1e9, ops / t / 1e12
    return {"bound": "hbm", "kernel": "int8 prefilter pass (v_mfma_i32_16x16x64_i8)",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "mfma_achieved_tops": round(tops, 1),
            "mfma_peak_tops": I8_DENSE_TOPS, "mfma_frac": round(tops / I8_DENSE_TOPS, 4),
            "bf16_equivalent_throughput_frac": round(tops / BF16_DENSE_TFLOPS, 4),
            "launches_per_step": -(-batch // per_launch), "kernel_ms": round(t_ms, 4),
            "bytes_per_launch": int(bytes_), "ops_per_launch": int(ops)}


def q8_gemv_roofline(rows_local, dim, k, t_ms):
    """One query on the int8 copy (r05): the scan launch streams
    the int8 rows (D bytes per row) and the query; HBM-bound. The rescore of
    the bracketed survivors (a few hundred rows) is its own, much shorter
    launch and is not priced here."""
    bytes_ = rows_local * dim + dim * 4 + k * 12
    t = t_ms / 1e3
    gbs = bytes_ / t / 1e9
    return {"bound": "hbm", "kernel": "int8 single-query scan (v_dot4_i32_i8)",
            "achieved": round(gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(gbs / HBM_PEAK_GBS, 4), "kernel_ms": round(t_ms, 4),
            "bytes_per_launch": int(bytes_)}


def q8_gemv_used(prefilter_bytes, dim, k):
    """Whether a one-query search takes the int8 copy (the engine's rule in
    vs_engine.cpp q8_gemv_path: a copy exists, dim 768 / 1024, k <= 128,
    VS_Q8_GEMV not 0)."""
    return (prefilter_bytes > 0 and dim in (768, 1024) and 1 <= k <= 128
            and os.environ.get("VS_Q8_GEMV", "1") != "0")


def pmc_traffic(workload, rows):
    """HBM bytes per launch from a committed rocprofv3 --pmc pass (profiles/),
    or None. An entry describes ONE launch over a given number of rows (its
    `rows`, the measured run's rows_per_gpu): it is reported only for a run
    whose rank scans exactly that many rows (key `<workload>@<rows>` or the
    plain `<workload>` entry when its rows match), never scaled to another
    share -- an N = 8 line must not carry the N = 1 launch's bytes."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        d = json.load(open(p))
    except Exception:
        return None
    for key in (f"{workload}@{rows}", workload):
        e = d.get(key)
        if isinstance(e, dict) and e.get("rows") == rows:
            return e.get("hbm_bytes_per_launch")
    return None


def queries_per_pass(dim, dtype):
    """Queries per launch of the bf16 / f32 MFMA pass."""
    return 256 if (dtype == "bf16" and dim <= 768) or (dtype == "f32" and dim <= 384) else 128


def scan_roofline(config, rows_local, dim, dtype, batch, k, scan_ms, int8, q8_b1=False):
    """The bench line's `roofline` for the dominant kernel of this rank's
    scan over `rows_local` rows: algorithmic bytes (or flops) of one launch
    over the rank's share / its measured duration, and `traffic` = the PMC
    HBM bytes of a launch over exactly that share (null when none was
    measured at that size)."""
    elem = 2 if dtype == "bf16" else 4
    if not scan_ms > 0:  # no scan launch was bracketed (never with the sampling rule above)
        return {"bound": "hbm" if (int8 or q8_b1 or batch == 1) else "mfma", "achieved": None,
                "peak": None, "unit": None, "frac": None, "traffic": None, "traffic_rows": None,
                "note": "no scan launch was timed"}
    if q8_b1:  # one query on the int8 copy
        roof = q8_gemv_roofline(rows_local, dim, k, scan_ms)
        roof["traffic"] = pmc_traffic(config + "_i8", rows_local)
        roof["traffic_rows"] = rows_local if roof["traffic"] is not None else None
        return roof
    if int8:  # the int8 pass takes 256 queries a launch up to 768-d, 128 above
        roof = int8_roofline(rows_local, dim, batch, k, scan_ms, 256 if dim <= 768 else 128)
    else:
        roof = kernel_roofline(rows_local, dim, elem, batch, k, scan_ms,
                               "mfma" if batch > 1 else "hbm", queries_per_pass(dim, dtype))
    roof["traffic"] = pmc_traffic(config + ("_i8" if int8 else ""), rows_local)
    roof["traffic_rows"] = rows_local if roof["traffic"] is not None else None
    return roof


def run_phase(eng, sharded, coll, dim, batch, k, steps, warmup, dist_on, stream_fn, row0,
              spec_coll=None):
    """Times `steps` searches; returns (max elapsed s over ranks, scan/merge ms,
    every timed step's result tensor, the query rows of each timed step).

    Every step searches a FRESH batch (r06): warmup +
    steps distinct batches of the query stream (query rows row0 + i * batch
    ...) are generated into HBM before the timer, and step i searches batch i,
    so nothing the engine learned from one batch (the speculative bound's
    ratio) is ever timed on the batch it was learned from. The
    result tensors rotate over at least `steps` buffers
    (shard.engine_callables ring), so each step's answer is still intact
    after the timed region."""
    import torch.distributed as dist

    nb = warmup + steps
    q = torch.empty((nb, batch, dim), dtype=torch.float32, device="cuda")
    eng.generate_vectors(0xC0FFEE, row0, nb * batch, dim, q.data_ptr(), stream_fn())
    for i in range(warmup):
        sharded.search(q[i], k)
    torch.cuda.synchronize()
    eng.timing(reset=True)
    # the speculative bound's counters over the timed steps only (read outside
    # the timer: the call waits for the device)
    spec0 = eng.spec_stats(spec_coll) if spec_coll else None
    if dist_on:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    outs = []
    for i in range(warmup, nb):
        outs.append(sharded.search(q[i], k))
    torch.cuda.synchronize()
    if dist_on:
        dist.barrier()
    el = time.perf_counter() - t0
    if dist_on:
        gloo = dist.get_backend() == "gloo"
        t = torch.tensor([el], dtype=torch.float64, device="cpu" if gloo else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    tm = eng.timing(reset=True)
    if spec_coll:
        s1 = eng.spec_stats(spec_coll)
        tm["spec"] = {key: s1[key] - spec0[key] for key in s1}
    return el, tm, outs, (q, warmup)


def verify_steps(pkg, outs, k, n_rows, sharded=None, qs=None, recheck=(0, -1)):
    """After the timed region: every timed step's answer is full (min(k, rows)
    keys per query) and sorted, and (with `sharded`) the steps in `recheck`,
    searched again on their own batch, return the same keys -- the answer
    does not depend on what the engine learned between. Raises on any
    violation; returns the checked count."""
    for o in outs:
        s, r, c = pkg.keys_decode(o.cpu().numpy().view(np.uint64))
        if int(c.min()) != min(k, n_rows):
            raise AssertionError("incomplete result lists")
        if not np.all(np.diff(s, axis=1) <= 0):
            raise AssertionError("unsorted results")
    if sharded is not None and qs is not None:
        q, w = qs
        for i in recheck:
            i = i % len(outs)
            again = sharded.search(q[w + i], k)
            torch.cuda.synchronize()
            if not np.array_equal(again.cpu().numpy(), outs[i].cpu().numpy()):
                raise AssertionError(f"timed step {i}: a second search of its batch differs")
    return len(outs)


def oracle_parity(pkg, cfg, n_full, outs, batch, row0, picks):
    """Part of the CPU-baseline leg (rank 0, N = 1): queries of several timed
    batches (`picks`: (step, query) pairs) checked against the streaming fp64
    oracle over the whole generated corpus (the north_star rule,
    oracle.check_topk). Test infrastructure only: called after the timed
    region, never timed."""
    from oracle import oracle

    rows, dim, dtype, metric, _, k, _ = cfg
    bf16 = dtype == "bf16"
    picks = [(st % len(outs), qi) for st, qi in picks if qi < batch]
    gids = [row0 + st * batch + qi for st, qi in picks]
    Q = np.concatenate([oracle.generate(oracle.SEED_QUERY, g, 1, dim) for g in gids])
    Qp = oracle.preprocess(Q, metric == "cosine", bf16)
    keys = np.stack([outs[st].cpu().numpy().view(np.uint64)[qi] for st, qi in picks])
    s, r, c = pkg.keys_decode(keys)
    t0 = time.perf_counter()
    s64, rr, cc = oracle.search_generated(oracle.SEED_CORPUS, 0, n_full, Qp, k, bf16)
    resc = oracle.rescore_generated(oracle.SEED_CORPUS, Qp, r, c, bf16)
    bad = oracle.check_topk(s, r, c, s64, rr, cc, resc, score_rtol=1e-5)
    return {"queries_checked": len(picks), "steps_and_queries": [list(p) for p in picks],
            "query_stream_rows": gids, "violations": len(bad), "first_violations": bad[:3],
            "rule": "north_star: ids exact except exact-score near-ties < 1e-5 rel; scores within "
                    "1e-5 rel of the fp64 score",
            "oracle": "oracle.search_generated (fp64, full corpus regenerated)",
            "oracle_s": round(time.perf_counter() - t0, 2)}


def cgroup_cpu_quota():
    """CPUs granted by the cgroup v2 CPU quota (cpu.max "quota period"), or None."""
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else max(1, int(int(q) // int(p)))
    except Exception:
        return None


def cpu_threads():
    """Threads for the CPU baseline: every CPU this process may run on
    (sched_getaffinity), capped by the cgroup CPU quota when one is set (more
    threads than the quota grants only queue on it). OMP_NUM_THREADS is
    recorded, not obeyed: the box sets it to its per-GPU worker share."""
    aff = len(os.sched_getaffinity(0))
    quota = cgroup_cpu_quota()
    n = min(aff, quota) if quota else aff
    return n, {"affinity_cpus": aff, "cgroup_quota_cpus": quota,
               "omp_num_threads_env": os.environ.get("OMP_NUM_THREADS")}


def cpu_blas_batched(X_raw, bf16, Q, k, threads, budget_s):
    """Batched CPU secondary: the batch's queries against row blocks as one
    fp32 GEMM each (torch CPU -> BLAS sgemm; bf16 rows widened per block),
    then a per-block top-k merged into the running top-k. Returns (queries/s
    over the full corpus, rows actually scanned, seconds)."""
    torch.set_num_threads(threads)
    n = X_raw.shape[0]
    q = torch.from_numpy(np.ascontiguousarray(Q, np.float32))
    blk = 8192  # fp32 blocks that stay in L3 between the widening and the GEMM
    best_s = torch.full((q.shape[0], k), -float("inf"))
    best_r = torch.zeros((q.shape[0], k), dtype=torch.int64)
    t0 = time.perf_counter()
    done = 0
    while done < n:
        xb = torch.from_numpy(X_raw[done:done + blk])
        xf = xb.view(torch.bfloat16).float() if bf16 else xb
        sc = q @ xf.T
        v, i = torch.topk(sc, min(k, sc.shape[1]), dim=1)
        best_s, j = torch.topk(torch.cat([best_s, v], 1), k, dim=1)
        best_r = torch.gather(torch.cat([best_r, i + done], 1), 1, j)
        done += xb.shape[0]
        if time.perf_counter() - t0 > budget_s and done >= n // 10:
            break
    el = time.perf_counter() - t0
    return q.shape[0] / (el * n / done), done, el


def cpu_baseline(cfg, args, n_full):
    """CPU baselines on this host (rank 0, N = 1), over the corpus the GPU
    searched (regenerated bit-identically on the host by the oracle's
    generator): (1) the oracle's Qdrant-style exact scan, one query at a time
    over the whole corpus, OpenMP over rows, AVX-512 build when the CPU has
    it; as many queries as fit the time budget (>= 4); (2) a batched BLAS
    secondary for the config's batch. Both report queries/s over the full
    corpus; a leg that stops early (budget) says how far it got."""
    from oracle import oracle

    rows, dim, dtype, metric, batch, k, _ = cfg
    bf16 = dtype == "bf16"
    ns = n_full if args.cpu_sample_rows <= 0 else min(args.cpu_sample_rows, n_full)
    threads, grant = cpu_threads()
    info = oracle.cpu_info()
    t0 = time.perf_counter()
    X = oracle.generate_raw(oracle.SEED_CORPUS, 0, ns, dim, bf16)
    gen_s = time.perf_counter() - t0
    Q = oracle.generate(oracle.SEED_QUERY, 0, max(batch, 64), dim, bf16=bf16)
    if metric == "cosine":
        Q = oracle.preprocess(Q, True, False)
    oracle.cpu_scan(X, bf16, Q[:1], k, threads=threads)  # warm (page-in)
    t0 = time.perf_counter()
    nq = 0
    nth = threads
    while nq < Q.shape[0] and (nq < 4 or time.perf_counter() - t0 < args.cpu_budget_s):
        _, _, nth = oracle.cpu_scan(X, bf16, Q[nq:nq + 2], k, threads=threads)
        nq += 2
    el = time.perf_counter() - t0
    qps = nq / (el * (n_full / ns))
    scope = (f"the full {n_full:,}-row corpus" if ns == n_full else
             f"the first {ns:,} of {n_full:,} rows (QPS scaled by {n_full / ns:.2f})")
    out = {"value": round(qps, 3), "unit": "queries/s", "cores": int(nth), "kind": "port",
           "sample": f"{nq} queries, one at a time (Qdrant-style scan), over {scope} "
                     f"({dtype}, dim {dim}, top-{k}); {el:.2f} s measured",
           "measured_s": round(el, 3), "isa": oracle.cpu_scan_isa(),
           "cpu_model": info["model"], "host_logical_cpus": info["logical_cpus"],
           "corpus_generate_s": round(gen_s, 2), "threads_grant": grant}
    if batch > 1:
        qps_b, done, el_b = cpu_blas_batched(X, bf16, Q[:batch], k, threads, args.cpu_budget_s)
        part = "" if done >= ns else f" (stopped at {done:,} rows by the budget; scaled)"
        out["batched"] = {
            "value": round(qps_b * ns / n_full, 3), "unit": "queries/s", "cores": threads,
            "method": "one fp32 GEMM per 8192-row block for the whole batch (torch CPU -> BLAS "
                      "sgemm, bf16 widened per block) + top-k merge",
            "sample": f"one {batch}-query batch over {scope}{part}; {el_b:.2f} s measured",
            "measured_s": round(el_b, 3)}
    return out


def main():
    args = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # VS_DIST_BACKEND=gloo (tests only): several ranks may then share one GPU
    # (RCCL refuses duplicate devices); the driver's runs use nccl = RCCL
    backend = os.environ.get("VS_DIST_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
    torch.cuda.set_device(local)
    # VS_BENCH_FORCE_DIST=1 (tests): the process group and the all-gather run
    # even with one rank, so the RCCL path is exercised on a one-GPU box
    force_dist = os.environ.get("VS_BENCH_FORCE_DIST") == "1"
    dist_on = world > 1 or force_dist
    if dist_on:
        import torch.distributed as dist
        if backend == "gloo":
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import __graft_entry__ as ge
    pkg = ge.load_package()
    from importlib import import_module
    shard = import_module(pkg.__name__ + ".shard")

    cfg = CONFIGS[args.config]
    n_full, dim, dtype, metric, batch, k, desc = cfg
    if args.rows:
        n_full = args.rows
    desc = desc.format(rows=fmt_rows(n_full))
    if args.rows:
        desc += " (--rows override of the config's corpus size)"
    lo, hi = shard.shard_range(n_full, world, rank)
    # the scans' event pairs: one launch in 4 (batches) / 16 (one query), the
    # 4th / 16th first (vsearch.h VS_FLAG_TIMING_SAMPLE); a run of fewer than
    # 16 timed steps brackets every scan, so it still times some
    sample = args.steps >= 16
    eng = pkg.VectorEngine(device=local, timing=True, timing_sample=sample)
    coll = "bench"
    eng.create_collection(coll, dim, pkg.METRIC_DOT if metric == "dot" else pkg.METRIC_COSINE,
                          pkg.DTYPE_BF16 if dtype == "bf16" else pkg.DTYPE_F32, hi - lo, lo)
    t0 = time.perf_counter()
    eng.generate(coll, hi - lo, 0x5EED)
    log(f"[bench] rank {rank}/{world}: rows [{lo}, {hi}) generated in "
        f"{time.perf_counter() - t0:.2f}s on {torch.cuda.get_device_name(local)}")

    stream_fn = lambda: torch.cuda.current_stream().cuda_stream  # noqa: E731
    # every timed step keeps its own result buffer (checked after the timer)
    ring = max(args.steps, 160)  # >= every phase's timed steps (the single-query line: 160)
    ls, mg = shard.engine_callables(eng, coll, dim, stream_fn, reuse=True, ring=ring)
    sharded = shard.ShardedSearch(ls, mg, always_gather=force_dist)
    # the data-path exchange: the engine's own RCCL communicator (all-gather +
    # merge on the search's stream) unless VS_COLLECTIVE=torch; gloo runs
    # (tests) always use torch.distributed
    collective = None
    if dist_on:
        collective = "gloo" if backend == "gloo" else os.environ.get("VS_COLLECTIVE", "engine")
        if collective == "engine":
            # every rank reaches each collective below whatever failed before
            # it; if any rank could not join, all keep torch's exchange
            uid = [None]
            if rank == 0:
                try:
                    uid = [pkg.VectorEngine.comm_unique_id()]
                except Exception as e:  # noqa: BLE001
                    log(f"[bench] rank 0: no RCCL unique id ({e})")
            dist.broadcast_object_list(uid, src=0)
            ok = 0
            if uid[0] is not None:
                try:
                    eng.comm_init(world, rank, uid[0])
                    ok = 1
                except Exception as e:  # noqa: BLE001
                    log(f"[bench] rank {rank}: engine communicator failed ({e})")
            flag = torch.tensor([ok], dtype=torch.int32, device="cuda")
            dist.all_reduce(flag, op=dist.ReduceOp.MIN)
            if int(flag.item()) == 1:
                sharded.gather_merge = shard.engine_gather_merge(eng, stream_fn, reuse=True,
                                                                 ring=ring)
                sharded.world_size = world
                # VS_EXCHANGE_OVERLAP=1: batch i's exchange on a stream of its own,
                # overlapping batch i + 1's search. Off by default: at the 1.25M
                # share it measured slower than the search stream (0.329 vs
                # 0.322 ms/step, profiles/r05_exchange_overlap.jsonl) -- the
                # RCCL and merge workgroups hold CUs the next sample pass needs
                if os.environ.get("VS_EXCHANGE_OVERLAP", "0") == "1":
                    sharded.exchange_stream = torch.cuda.Stream()
                    sharded.exchange_ring = ring
            else:
                log("[bench] torch.distributed exchange instead of the engine communicator")
                collective = "torch"

    int8_pre = batch > 1 and eng.prefilter_bytes(coll) > 0
    el, tm, outs, qs = run_phase(eng, sharded, coll, dim, batch, k, args.steps, args.warmup,
                                 dist_on, stream_fn, 0, coll if int8_pre else None)
    spec = tm.get("spec")
    out = outs[-1]
    steps_verified = verify_steps(pkg, outs, k, n_full, sharded, qs)
    elem = 2 if dtype == "bf16" else 4
    # batched bf16 searches of a collection with an int8 copy run the int8
    # prefilter pass (the engine's default; VS_FLAG_NO_PREFILTER turns it off)
    int8 = int8_pre
    q8_b1 = batch == 1 and q8_gemv_used(eng.prefilter_bytes(coll), dim, k)
    qpp = queries_per_pass(dim, dtype)
    roof = scan_roofline(args.config, hi - lo, dim, dtype, batch, k, tm["scan_ms"], int8, q8_b1)
    roof["kernel_launches_timed"] = tm["scan_n"]

    result = {
        "metric": METRIC_NAME,
        "value": round(batch * args.steps / el, 2),
        "unit": "queries/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(el / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        # int8 pass + rescoring of its survivors on the bf16 / f32 pass's chain
        "dtype": f"i8+{dtype}" if (int8 or q8_b1) else dtype,
        "data": "synthetic (counter-based unit-norm generator, seeds 0x5EED / 0xC0FFEE)",
        "config": {"workload": desc, "corpus_rows": n_full, "dim": dim, "batch": batch, "k": k,
                   "metric": metric, "parallelism": f"row-shard x{world}",
                   "rows_per_gpu": hi - lo, "collective": collective,
                   "exchange_overlapped": sharded.exchange_stream is not None,
                   "int8_prefilter": int8, "int8_single_query": q8_b1,
                   # (r05) batches after the first start from the collection's
                   # learned k-th-score ratio, checked per query in the select,
                   # the sample path re-run on a miss
                   "int8_speculative_bound": bool(int8 and batch > 1
                                                  and os.environ.get("VS_Q8_SPEC", "1") != "0"),
                   "build_id": pkg.build_id()},
        "roofline": roof,
        "steps_verified": steps_verified,
        # (r06) each timed step searched its own fresh batch; speculative
        # batches of the timed steps whose check failed (the sample path then
        # re-answered them), and those a cool-down sent to the sample path
        "fresh_batches": True,
        "spec_fallbacks": spec["fallbacks"] if spec else None,
        "spec_stats": spec,
    }

    # secondary: the single-query GEMV line on the same resident corpus
    if not args.no_secondary and batch > 1:
        # 160+ single-query steps after 10 of warmup: at ~1.3 ms each the line
        # costs a fifth of a second, and its sampled kernel average (every 16th
        # launch) rests on 10+ launches
        steps1 = max(160, args.steps)
        el1, tm1, outs1, qs1 = run_phase(eng, sharded, coll, dim, 1, k, steps1, 10, dist_on,
                                         stream_fn, 1000)
        r1 = scan_roofline(args.config + "b1", hi - lo, dim, dtype, 1, k, tm1["scan_ms"], False,
                           q8_gemv_used(eng.prefilter_bytes(coll), dim, k))
        result["secondary"] = {"workload": "same corpus, single query (GEMV path)",
                               "value": round(steps1 / el1, 2), "unit": "queries/s",
                               "ms_per_step": round(el1 / steps1 * 1e3, 4), "roofline": r1,
                               "steps_verified": verify_steps(pkg, outs1, k, n_full, sharded,
                                                              qs1)}

    # secondary (one GPU): the same batch on the bf16 / f32 pass alone -- a
    # second engine without the int8 copy over the same generated rows
    if int8 and world == 1 and not dist_on and not args.no_secondary:
        eng.drop_collection(coll)  # room for the second corpus
        e2 = pkg.VectorEngine(device=local, timing=True, timing_sample=sample, prefilter=False)
        try:
            e2.create_collection(coll, dim, pkg.METRIC_DOT if metric == "dot" else
                                 pkg.METRIC_COSINE,
                                 pkg.DTYPE_BF16 if dtype == "bf16" else pkg.DTYPE_F32, hi - lo, lo)
            e2.generate(coll, hi - lo, 0x5EED)
            ls2, mg2 = shard.engine_callables(e2, coll, dim, stream_fn, reuse=True, ring=ring)
            sh2 = shard.ShardedSearch(ls2, mg2)
            el2, tm2, outs2, _ = run_phase(e2, sh2, coll, dim, batch, k, args.steps, args.warmup,
                                           False, stream_fn, 0)
            # the int8 path rescores on the bf16 pass's MFMA chain: same keys,
            # every timed step (the same fresh batches in the same order)
            same = float(np.mean([(a.cpu().numpy().view(np.uint64) ==
                                   b.cpu().numpy().view(np.uint64)).mean()
                                  for a, b in zip(outs2, outs)]))
            result[f"{dtype}_pass"] = {
                "workload": f"the same batch on the {dtype} MFMA pass (VS_FLAG_NO_PREFILTER)",
                "value": round(batch * args.steps / el2, 2), "unit": "queries/s",
                "ms_per_step": round(el2 / args.steps * 1e3, 4),
                "roofline": kernel_roofline(hi - lo, dim, elem, batch, k, tm2["scan_ms"], "mfma", qpp),
                "steps_verified": verify_steps(pkg, outs2, k, n_full),
                "keys_equal_to_int8_path": round(same, 6)}
        finally:
            e2.close()

    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            result["cpu_baseline"] = cpu_baseline(cfg, args, n_full)
        except Exception as e:  # the baseline never decides the run
            result["cpu_baseline"] = {"value": None, "error": repr(e)}
        # the same leg checks the timed batch against the oracle (outside the timer)
        try:
            K = len(outs)
            result["parity"] = oracle_parity(pkg, cfg, n_full, outs, batch, args.warmup * batch,
                                             [(0, 0), (K // 3, 85), (2 * K // 3, 170),
                                              (K - 1, 255)])
        except Exception as e:  # reported, never silent
            result["parity"] = {"queries_checked": 0, "error": repr(e)}
    elif rank == 0:
        result["cpu_baseline"] = None

    if rank == 0 and args.dump_keys:
        np.save(args.dump_keys, out.cpu().numpy().view(np.uint64))

    if rank == 0:
        print(json.dumps(result), flush=True)
    eng.close()
    if dist_on:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
