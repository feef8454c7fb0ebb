import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
eng = pkg.VectorEngine(device=0)
n = 64
eng.create_collection("a", 768, 0, 1); eng.generate("a", n, orc.SEED_CORPUS)
eng.create_collection("lo", 768, 0, 1, 0, 0); eng.generate("lo", 32, orc.SEED_CORPUS)
eng.create_collection("hi", 768, 0, 1, 0, 32); eng.generate("hi", 32, orc.SEED_CORPUS)
X = orc.generate(orc.SEED_CORPUS, 0, n, 768, True)
Q = orc.generate(orc.SEED_QUERY, 0, 32, 768)
Qp = orc.preprocess(Q, True, True)
S = Qp.astype(np.float64) @ X.astype(np.float64).T
for k in (1, 2, 3, 4, 10):
    s, r, c = eng.search("a", Q, k)
    ref = np.argsort(-S, axis=1, kind="stable")[:, :k]
    bad = [i for i in range(32) if r[i].tolist() != ref[i].tolist()]
    print("k", k, "bad queries", bad)
for nm, off in (("lo", 0), ("hi", 32)):
    s, r, c = eng.search(nm, Q, 1)
    ref = np.argmax(S[:, off:off + 32], axis=1) + off
    print(nm, "bad", [i for i in range(32) if r[i, 0] != ref[i]])
    s, r, c = eng.search(nm, Q, 2)
    ref2 = np.argsort(-S[:, off:off + 32], axis=1, kind="stable")[:, :2] + off
    print(nm, "k2 bad", [i for i in range(32) if r[i].tolist() != ref2[i].tolist()])
    # detail for q2
    print(nm, "q2 dev", r[2].tolist(), s[2].tolist(), "ref", ref2[2].tolist(), S[2, ref2[2]].tolist())
    top = np.argsort(-S[2, off:off+32])[:5] + off
    print(nm, "q2 top5 rows", top.tolist(), S[2, top].round(5).tolist())
