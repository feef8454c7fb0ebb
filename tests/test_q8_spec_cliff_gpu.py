"""The speculative bound under off-topic queries (r06).

r05's ratio was one running minimum over every verified query, so a single
query whose k-th score is far under the rest (an off-topic question against
clustered embeddings: the traffic retrieval-service sends one query at a
time, rag/retrieval-service/main.go:219-276) pinned the bound of every later
batch near zero until the next write: the answers stayed exact, the int8 pass
then admitted whole clusters. Now a batch REPLACES the ratio with a low
quantile of its own queries' ratios (csrc/vs_q8.hip q8_verify_record_kernel)
and a failed check backs off to the sample path.

Two corpora (4M unit rows, bf16, inner product): 64 Gaussian clusters, where
one ratio cannot follow the queries' own k-th scores and speculation must
switch itself off (Q8SpecK.loose), and isotropic rows with planted topics of
near-duplicates, where it pays and must keep paying. Each is searched in one
process by two engines over the same rows: speculation on (the default) and
off (VS_FLAG_NO_SPECULATIVE, the sample path every batch).
The sequence: on-topic batches (the ratio is learned), ONE batch mixing
on-topic queries with a few near-orthogonal ones, then more fresh on-topic
batches, then a run of batches that all carry outliers. Checked: keys
bit-identical between the engines on every batch, the oracle on the outliers
and on on-topic queries after them, and -- the point -- no on-topic batch
after the outlier runs more than 2% slower with speculation on than off
(relative to the engines' ratio on identical sample-path work, measured
first: it absorbs a per-engine memory-placement difference, 3.5% on one box)
(device events around each batch; each fresh batch runs once on each of two
speculating engines fed the same batches in the same order -- replicas of one
state -- interleaved with two runs of the stateless one, and the faster of
each pair is compared, so a one-run stall on either side cancels).
Anchor: Points.Search, rag/vector-service/main.go:249-254.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

_CLIFF = r"""
import sys, os, json
sys.path.insert(0, ROOT)
import numpy as np
import torch
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
n, dim, C, B, k = int(os.environ.get("T_ROWS", "4000000")), 768, 64, 256, 10
g = torch.Generator(device="cuda").manual_seed(2026)
cent = torch.randn((C, dim), device="cuda", generator=g)
cent /= cent.norm(dim=1, keepdim=True)
KIND = os.environ.get("T_KIND", "clusters")
def unit(v):
    return v / v.norm(dim=1, keepdim=True)
if KIND == "clusters":
    # 64 Gaussian clusters: every row and on-topic query is a centre plus noise
    # of the same norm, so a query's own cluster crowds the scores just under
    # its k-th, and that k-th moves with the query (its noise along the centre)
    def clustered(m, noise=1.0):
        lab = torch.randint(0, C, (m,), device="cuda", generator=g)
        return unit(cent[lab] + noise * torch.randn((m, dim), device="cuda", generator=g) / dim ** 0.5)
    X = torch.cat([clustered(200_000) for _ in range(n // 200_000)]).cpu().numpy()
    # near-orthogonal to every cluster centre: the centres' span projected out
    Qc, _ = torch.linalg.qr(cent.T)
    def outliers(m):
        v = torch.randn((m, dim), device="cuda", generator=g)
        return unit(v - (v @ Qc) @ Qc.T)
else:
    # "planted": isotropic random rows plus 4096 topics of 32 near-duplicate
    # rows each (RAG chunks close to a question); an on-topic query sits on a
    # topic (k-th score ~0.9), an outlier is a random direction (~0.16)
    T, per = 4096, 32
    top = unit(torch.randn((T, dim), device="cuda", generator=g))
    def near(t, m):
        return unit(top[t] + 0.35 * torch.randn((m, dim), device="cuda", generator=g) / dim ** 0.5)
    Xt = torch.empty((n, dim), device="cuda")
    for r0 in range(0, n, 200_000):
        r1 = min(n, r0 + 200_000)
        Xt[r0:r1] = unit(torch.randn((r1 - r0, dim), device="cuda", generator=g))
    slots = torch.randperm(n, device="cuda", generator=g)[:T * per]
    Xt[slots] = near(torch.arange(T, device="cuda").repeat_interleave(per), T * per)
    X = Xt.cpu().numpy()
    del Xt
    def clustered(m):
        return near(torch.randint(0, T, (m,), device="cuda", generator=g), m)
    def outliers(m):
        return unit(torch.randn((m, dim), device="cuda", generator=g))
if os.environ.get("T_OFF_FIRST") == "1":
    off = pkg.VectorEngine(device=0, speculative=False)
on = pkg.VectorEngine(device=0)
on2 = pkg.VectorEngine(device=0)  # the same batches in the same order: a replica of on
if os.environ.get("T_OFF_FIRST") != "1":
    off = pkg.VectorEngine(device=0, speculative=False)
order = (off, on, on2) if os.environ.get("T_OFF_FIRST") == "1" else (on, on2, off)
for e in order:
    e.create_collection("c", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
    for r0 in range(0, n, 500_000):
        e.upsert("c", np.arange(r0, min(n, r0 + 500_000), dtype=np.uint64), X[r0:r0 + 500_000])
assert on.prefilter_bytes("c") > 0
stream = torch.cuda.current_stream()
keys = {e: torch.empty((B, k), dtype=torch.int64, device="cuda") for e in (on, on2, off)}
ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
def run(e, q, kk=k):
    ev[0].record(stream)
    e.search_keys("c", q.data_ptr(), B, dim, kk, keys[e].data_ptr(), stream.cuda_stream)
    ev[1].record(stream)
    ev[1].synchronize()
    return (ev[0].elapsed_time(ev[1]),
            keys[e].cpu().numpy().view(np.uint64).reshape(-1)[:B * kk].reshape(B, kk).copy())
out = {"batches": [], "mismatch": [], "parity": [], "stats": {}}
kept = []  # (phase, queries, keys) for the oracle
def batch(phase, q, kk=k):
    # each speculating engine runs each fresh batch ONCE (on and on2 keep one
    # state between them: never a batch learned from itself), interleaved with
    # two runs of the stateless engine; the faster run of each side counts, so
    # a one-run stall on either side cancels and clock drift is bracketed
    i = len(out["batches"])
    t0, k0 = run(off, q, kk)
    t1, k1 = run(on, q, kk)
    t2, _ = run(off, q, kk)
    t3, k3 = run(on2, q, kk)
    if not (np.array_equal(k1, k0) and np.array_equal(k3, k0)):
        out["mismatch"].append(i)
    out["batches"].append({"phase": phase, "on_ms": min(t1, t3), "off_ms": min(t0, t2),
                           "on_runs_ms": [t1, t3], "off_runs_ms": [t0, t2]})
    return k1
# calibration: the engines' relative speed on identical work. A batch of a k
# no context has answered yet runs the sample path on both engines (k = 1 ..
# 9 rising: a k' >= k seen is what a speculative try needs, and none of these
# is ever >= 10), so its ratio is the engines' memory placement, not
# speculation (one box read 1.035 on every such batch, r06)
for kk in range(1, 10):
    batch("calib", clustered(B), kk)
# warm both engines and the learned ratio on on-topic batches
for _ in range(6):
    batch("warm", clustered(B))
# one batch with a few off-topic queries among on-topic ones
nout = int(os.environ.get("T_OUTLIERS", "3"))
q = torch.cat([clustered(B - nout), outliers(nout)])
kq = batch("outlier", q)
kept.append(("outlier", q[B - nout - 2:].cpu().numpy(), kq[B - nout - 2:]))
# fresh on-topic batches after it
for i in range(10):
    q = clustered(B)
    kq = batch("after", q)
    if i in (0, 5):
        kept.append(("after", q[:3].cpu().numpy(), kq[:3]))
# every batch carrying outliers (back-off regime)
for i in range(int(os.environ.get("T_MIXED", "16"))):
    q = torch.cat([clustered(B - nout), outliers(nout)])
    batch("mixed", q)
out["stats"] = {"on": on.spec_stats("c"), "on2": on2.spec_stats("c"), "off": off.spec_stats("c")}
# the oracle on the kept queries (rows as stored: bf16)
Xb = orc.preprocess(X, False, True)
for phase, Q, kk in kept:
    Q = orc.preprocess(Q, False, True)
    s, r, c = pkg.keys_decode(kk)
    _, s64, rr, cc = orc.search(Xb, Q, k)
    resc = orc.rescore(Xb, Q, r, c)
    bad = orc.check_topk(s, r, c, s64, rr, cc, resc, 1e-5)
    if bad:
        out["parity"].append([phase, bad[:3]])
on.close(); on2.close(); off.close()
print(json.dumps(out))
"""


def _run(env):
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, **env)
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % root + _CLIFF], env=e, cwd=root,
                       capture_output=True, text=True, timeout=900)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("kind", ["clusters", "planted"])
def test_outlier_queries_do_not_poison_later_batches(kind):
    r = _run({"T_KIND": kind})
    rec = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpurun_out")
    if os.path.isdir(rec):
        with open(os.path.join(rec, f"spec_cliff_{kind}.json"), "w") as f:
            json.dump(r, f)
    assert r["mismatch"] == [], r["mismatch"]
    assert r["parity"] == [], r["parity"]
    b = r["batches"]
    # the engines' relative speed on identical (sample-path) work: every ratio
    # below is taken relative to it
    # (the low end, not the median: the first run of each k on each engine
    # grows its scratch -- a synchronize and an allocation -- which both
    # speculating engines' only run pays and the stateless engine's second run
    # does not, so that term only ever inflates a calibration ratio; r06h:
    # 3 of 9 read 1.07-1.34 beside 1.004-1.039)
    cal = sorted(x["on_ms"] / x["off_ms"] for x in b if x["phase"] == "calib")
    r0 = cal[1]
    assert 0.9 <= r0 <= 1.1, cal
    after = [x for x in b if x["phase"] == "after"]
    # single-batch times jitter by ~1-2% on the same work, so each ratio is
    # over a pair of consecutive fresh batches
    ratios = [(after[i]["on_ms"] + after[i + 1]["on_ms"]) /
              (after[i]["off_ms"] + after[i + 1]["off_ms"]) / r0 for i in range(len(after) - 1)]
    # no on-topic batch after the outlier pays for it (r05's running minimum
    # made every one of them several times slower)
    assert max(ratios) <= 1.02, ratios
    st = r["stats"]["on"]
    assert r["stats"]["on2"] == st, r["stats"]  # the replica took the same decisions
    assert r["stats"]["off"]["tries"] == 0, r["stats"]
    mixed = [x for x in b if x["phase"] == "mixed"]
    tail = mixed[len(mixed) // 2:]
    assert sum(x["on_ms"] for x in tail) <= 1.25 * r0 * sum(x["off_ms"] for x in tail), tail
    if kind == "planted":
        # a corpus where speculating pays: it kept paying after the outlier
        # (the outlier failed its batch's check; the ratio it would have
        # dragged down was never learned), and every-batch outliers backed off
        assert sorted(ratios)[len(ratios) // 2] <= 0.95, ratios
        assert st["fallbacks"] >= 1 and st["skipped"] >= 1, st
