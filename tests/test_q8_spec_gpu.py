"""Speculative bound on the int8 path (r05; DESIGN.md §5 "Speculative bound",
csrc/vs_engine.cpp search_mfma, csrc/vs_q8.hip q8_verify_record_kernel).

Once a search context has answered an unfiltered bf16 batch of a collection
at some k, later batches at k' <= k start the int8 pass from bound = ratio x
|q| (0.97 x the smallest verified k-th score per |q|) instead of a sample
pass. The answer is exact iff every query's k-th exact score reaches its
bound - sigma nmax; otherwise the whole batch re-runs on the sample path,
gated on that verdict on the device. Checked in a child process with one
search context (VS_CONTEXTS=1, so the second batch takes the speculative
path): repeated and fresh batches, smaller k, a write in between (the ratios
are reset), and every speculative batch forced to fail (the gated fallback
answers it) -- keys bit-identical to the plain bf16 pass every time, and to
the oracle. Anchor: Points.Search, rag/vector-service/main.go:249-254.
"""
import pytest

pytestmark = pytest.mark.gpu

_SPEC = r"""
import sys, json
sys.path.insert(0, ROOT)
import numpy as np
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
import os
n, dim = 200_000, int(os.environ.get("T_DIM", "768"))
cosine = os.environ.get("T_COSINE") == "1"
nq = int(os.environ.get("T_NQ", "256"))
ks = [int(x) for x in os.environ.get("T_KS", "10,10,10,10,5,50,50,50").split(",")]
f32 = os.environ.get("T_F32") == "1"
a = pkg.VectorEngine(device=0)
b = pkg.VectorEngine(device=0, prefilter=False)
for e in (a, b):
    e.create_collection("p", dim, pkg.METRIC_COSINE if cosine else pkg.METRIC_DOT,
                        pkg.DTYPE_F32 if f32 else pkg.DTYPE_BF16, n + 4096)
    e.generate("p", n, 91)
out = {"mismatch": [], "parity": []}
X = orc.generate(91, 0, n, dim, bf16=not f32)

def check(tag, Q, k):
    s1, r1, c1 = a.search("p", Q, k)
    s2, r2, c2 = b.search("p", Q, k)
    same = (np.array_equal(c1, c2) and np.array_equal(r1, r2)
            and np.array_equal(s1.view(np.uint32), s2.view(np.uint32)))
    if not same:
        out["mismatch"].append(tag)
    return s1, r1, c1

# batches: repeated, fresh, smaller and larger k (the KS list, in order)
q0s = [0, 0, 0, 1, 2, 3, 3, 4]
for i, k in enumerate(ks):
    Q = orc.generate(orc.SEED_QUERY, q0s[i % len(q0s)] * nq, nq, dim)
    check("batch%d_k%d" % (i, k), Q, k)
# a write in between: the ratios are reset, the next batch takes the sample path
rows = np.arange(0, 200, dtype=np.uint64) * 97
V = orc.generate(5, 0, 200, dim)
for e in (a, b):
    e.upsert("p", rows, V)
Q = orc.generate(orc.SEED_QUERY, 0, nq, dim)
k0 = ks[0]
for tag in ("after_write", "after_write_again"):
    check(tag, Q, k0)
# the oracle on the final rows, for the last batch
Xw = orc.preprocess(X, cosine, not f32) if cosine else X.copy()
Xw[rows.astype(np.int64)] = orc.preprocess(V, cosine, not f32)
Qp = orc.preprocess(Q, cosine, not f32)
s, r, c = a.search("p", Q, k0)
_, s64, rr, cc = orc.search(Xw, Qp, k0)
resc = orc.rescore(Xw, Qp, r, c)
out["parity"] = orc.check_topk(s, r, c, s64, rr, cc, resc, 1e-5)[:5]
a.close(); b.close()
print(json.dumps(out))
"""


def _run(env):
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, VS_CONTEXTS="1", **env)
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % root + _SPEC], env=e, cwd=root,
                       capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-3000:]
    return json.loads(p.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("env", [{}, {"VS_Q8_SPEC_FORCE_FAIL": "1"}, {"VS_Q8_SPEC": "0"}],
                         ids=["speculative", "forced_fallback", "off"])
def test_speculative_bound_keys_equal_bf16_pass(env):
    r = _run(env)
    assert r["mismatch"] == [], r["mismatch"]
    assert r["parity"] == [], r["parity"]


@pytest.mark.parametrize("env", [{}, {"VS_Q8_SPEC_FORCE_FAIL": "1"}], ids=["speculative", "forced_fallback"])
def test_speculative_bound_1024_cosine_two_chunks(env):
    """C5's row shape (1024-d cosine, 128 queries a launch), 300 queries a
    call (three int8 launches), k up to 128."""
    r = _run(dict(env, T_DIM="1024", T_COSINE="1", T_NQ="300", T_KS="128,128,7,128,40,100,128,3"))
    assert r["mismatch"] == [], r["mismatch"]
    assert r["parity"] == [], r["parity"]


@pytest.mark.parametrize("env", [{}, {"VS_Q8_SPEC_FORCE_FAIL": "1"}], ids=["speculative", "forced_fallback"])
def test_speculative_bound_fp32(env):
    """fp32 rows: two 128-query sample passes behind a speculative try (both
    gated), survivors rescored on the f32 pass's chain."""
    r = _run(dict(env, T_F32="1", T_KS="10,10,10,10,5,64,64,64"))
    assert r["mismatch"] == [], r["mismatch"]
    assert r["parity"] == [], r["parity"]


_NEG = r"""
import sys, json
sys.path.insert(0, ROOT)
import numpy as np
import __graft_entry__ as ge
pkg = ge.load_package()
n, dim, nq, k = 200_000, 768, 256, 10
rng = np.random.default_rng(5)
u = rng.standard_normal(dim).astype(np.float32)
u /= np.linalg.norm(u)
# every row points away from u (inner products all about -1), the queries
# along u: no batch has a k-th score > 0, so none records a ratio
X = -u[None, :] + 0.05 * rng.standard_normal((n, dim)).astype(np.float32) / dim ** 0.5
a = pkg.VectorEngine(device=0)
b = pkg.VectorEngine(device=0, prefilter=False)
for e in (a, b):
    e.create_collection("neg", dim, pkg.METRIC_DOT, pkg.DTYPE_BF16, n)
    e.upsert("neg", np.arange(n, dtype=np.uint64), X)
out = {"mismatch": []}
for i in range(4):
    Q = u[None, :] + 0.05 * rng.standard_normal((nq, dim)).astype(np.float32) / dim ** 0.5
    s1, r1, c1 = a.search("neg", Q, k)
    s2, r2, c2 = b.search("neg", Q, k)
    if not (np.array_equal(r1, r2) and np.array_equal(s1.view(np.uint32), s2.view(np.uint32))):
        out["mismatch"].append(i)
    out["max_kth"] = float(s1[:, k - 1].max())
out["stats"] = a.spec_stats("neg")
a.close(); b.close()
print(json.dumps(out))
"""


def test_no_positive_kth_never_speculates():
    """a dot collection whose k-th scores are all <= 0 records no
    ratio; the batches after its first must not run on an unset bound (r05
    ran them with bound = -inf: every row admitted). The device sees the
    ratio unset and stands the speculative launches down, so the sample path
    answers: keys equal the bf16 pass's, and no speculative batch is counted."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    e = dict(os.environ, VS_CONTEXTS="1")
    p = subprocess.run([sys.executable, "-c", "ROOT = %r\n" % root + _NEG], env=e, cwd=root,
                       capture_output=True, text=True, timeout=300)
    assert p.returncode == 0, p.stderr[-3000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["mismatch"] == [], r
    assert r["max_kth"] < 0, r
    assert r["stats"]["tries"] == 0 and r["stats"]["skipped"] >= 3, r["stats"]
