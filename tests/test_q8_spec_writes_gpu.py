"""Writes into the collection that speculative batches are searching (r06;
VERDICT r05 item 5, ADVICE r05: several search contexts).

The speculative bound's state is device memory shared by every search context
of a device (csrc/vs_kernels.h Q8SpecK, after the collection's int8 bounds);
a store-side write resets it on the writer's stream and bumps the copy's
generation (vs_engine.cpp q8_spec_reset), while other contexts' batches may
be reading or recording it. Exactness never rests on the ratio (every
speculative batch is checked), so the claim tested here is the whole one:
every answer equals the answer on the rows as they stood when its call took
the collection's reader lock.

In a child process with three search contexts (VS_CONTEXTS=3): two threads
issue host-API batched searches at mixed k (vs_search picks a context), one
thread issues device-pointer searches on its own stream (vs_search_keys, the
bench / shard path), and a writer overwrites scattered rows and appends rows
to THAT collection. Each call records the writes completed before it started
and the writes started before it returned; its keys must equal, bit for bit,
the keys of one version in that window, as computed afterwards by a second
engine without the int8 copy (the bf16 pass) to which the same writes are
replayed one by one; the final version's answers are checked against the
oracle. Anchors: concurrent handlers rag/vector-service/main.go:77, upsert
:149-225, Points.Search :249-254.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

_WRITES = r"""
import sys, os, json, threading
sys.path.insert(0, ROOT)
import numpy as np
import torch
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
n0, dim = 300_000, 768
# query sets: (queries' first stream row, nq, k); mixed k, one >256-query call
QS = [(0, 256, 10), (256, 256, 50), (512, 64, 128), (600, 300, 7), (1000, 256, 10)]
Qs = [orc.generate(orc.SEED_QUERY, r0, nq, dim) for r0, nq, _ in QS]
# the writes: scattered overwrites, then an append, alternately
rng = np.random.default_rng(11)
writes = []
rows_now = n0
for w in range(8):
    if w % 2 == 0:
        rows = np.unique(rng.integers(0, rows_now, 700)).astype(np.uint64)
    else:
        rows = np.arange(rows_now, rows_now + 4096, dtype=np.uint64)
        rows_now += 4096
    writes.append((rows, orc.generate(1234 + w, 0, len(rows), dim)))
a = pkg.VectorEngine(device=0)
a.create_collection("w", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, rows_now + 4096)
a.generate("w", n0, 77)
assert a.prefilter_bytes("w") > 0
started = [0]
done = [0]
lock = threading.Lock()
log = []  # (qset, lo, hi, keys)
errors = []
stop = threading.Event()

def record(qi, lo, keys):
    with lock:
        hi = started[0]
        log.append((qi, lo, hi, keys))

def host_searcher(seed):
    r = np.random.default_rng(seed)
    try:
        while not stop.is_set():
            qi = int(r.integers(0, len(QS)))
            lo = done[0]
            s, rr, c = a.search("w", Qs[qi], QS[qi][2])
            keys = np.stack([s.view(np.uint32).astype(np.uint64), rr, c.astype(np.uint64)[:, None]
                             .repeat(rr.shape[1], 1)])
            record(qi, lo, keys)
    except Exception as e:
        errors.append(("host", repr(e)))

def dev_searcher():
    try:
        st = torch.cuda.Stream()
        dq = [torch.from_numpy(Q).cuda() for Q in Qs]
        i = 0
        while not stop.is_set():
            qi = i % len(QS)
            i += 1
            nq, k = QS[qi][1], QS[qi][2]
            out = torch.empty((nq, k), dtype=torch.int64, device="cuda")
            lo = done[0]
            with torch.cuda.stream(st):
                a.search_keys("w", dq[qi].data_ptr(), nq, dim, k, out.data_ptr(), st.cuda_stream)
            with lock:
                hi = started[0]
            st.synchronize()
            s, rr, c = pkg.keys_decode(out.cpu().numpy().view(np.uint64))
            keys = np.stack([s.view(np.uint32).astype(np.uint64), rr, c.astype(np.uint64)[:, None]
                             .repeat(rr.shape[1], 1)])
            with lock:
                log.append((qi, lo, hi, keys))
    except Exception as e:
        errors.append(("device", repr(e)))

def writer():
    try:
        import time
        time.sleep(0.3)
        for rows, V in writes:
            with lock:
                started[0] += 1
            a.upsert("w", rows, V)
            done[0] += 1
            time.sleep(0.15)
    except Exception as e:
        errors.append(("write", repr(e)))

th = [threading.Thread(target=host_searcher, args=(s,)) for s in (1, 2)]
th += [threading.Thread(target=dev_searcher)]
wt = threading.Thread(target=writer)
for t in th + [wt]:
    t.start()
wt.join()
import time
time.sleep(0.3)
stop.set()
for t in th:
    t.join()
out = {"errors": errors, "calls": len(log), "bad": [], "per_version": {}, "parity": [],
       "spec": a.spec_stats("w")}
# every version's expected keys from a bf16-pass engine, the writes replayed
b = pkg.VectorEngine(device=0, prefilter=False)
b.create_collection("w", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, rows_now + 4096)
b.generate("w", n0, 77)
def answers():
    res = []
    for qi, (r0, nq, k) in enumerate(QS):
        s, rr, c = b.search("w", Qs[qi], k)
        res.append(np.stack([s.view(np.uint32).astype(np.uint64), rr,
                             c.astype(np.uint64)[:, None].repeat(rr.shape[1], 1)]))
    return res
expect = [answers()]
for rows, V in writes:
    b.upsert("w", rows, V)
    expect.append(answers())
for qi, lo, hi, keys in log:
    ok = [v for v in range(lo, min(hi, len(writes)) + 1) if np.array_equal(keys, expect[v][qi])]
    if not ok:
        out["bad"].append([qi, lo, hi])
    else:
        out["per_version"][str(ok[0])] = out["per_version"].get(str(ok[0]), 0) + 1
# the final version against the oracle (a few queries of each set)
X = orc.generate(77, 0, n0, dim, bf16=True)
X = np.concatenate([X, np.zeros((rows_now - n0, dim), np.float32)])
for rows, V in writes:
    X[rows.astype(np.int64)] = orc.preprocess(V, False, True)
for qi, (r0, nq, k) in enumerate(QS):
    Qp = orc.preprocess(Qs[qi][:4], False, True)
    s = expect[-1][qi][0][:4].astype(np.uint32).view(np.float32)
    r = expect[-1][qi][1][:4]
    c = expect[-1][qi][2][:4, 0].astype(np.uint32)
    _, s64, rr, cc = orc.search(X, Qp, k)
    bad = orc.check_topk(s, r, c, s64, rr, cc, orc.rescore(X, Qp, r, c), 1e-5)
    if bad:
        out["parity"].append([qi, bad[:2]])
a.close(); b.close()
print(json.dumps(out))
"""


def test_writes_into_the_searched_collection_across_contexts():
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, VS_CONTEXTS="3")
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % root + _WRITES], env=e, cwd=root,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["errors"] == [], r["errors"]
    assert r["bad"] == [], (r["bad"][:5], r["calls"])
    assert r["parity"] == [], r["parity"]
    # searches landed on several versions, and speculative batches ran
    assert len(r["per_version"]) >= 3, r["per_version"]
    assert r["spec"]["tries"] > 0, r["spec"]
