"""Focused parity probe for the batched MFMA scan (debug aid)."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import __graft_entry__ as ge
from oracle import oracle as orc
pkg = ge.load_package()
eng = pkg.VectorEngine(device=0)
for n in (32, 64, 4096, 8192, 20000):
    nm = f"d{n}"
    eng.create_collection(nm, 768, 0, 1)
    eng.generate(nm, n, orc.SEED_CORPUS)
    X = orc.generate(orc.SEED_CORPUS, 0, n, 768, True)
    for nq in (32, 256):
        Q = orc.generate(orc.SEED_QUERY, 0, nq, 768)
        Qp = orc.preprocess(Q, True, True)
        for k in (1, 10):
            s32, s64, rows, cnt = orc.search(X, Qp, k)
            res = []
            for rep in range(3):
                s, r, c = eng.search(nm, Q, k)
                resc = orc.rescore(X, Qp, r, c)
                bad = orc.check_topk(s, r, c, s64, rows, cnt, resc, 1e-5)
                res.append(len(bad))
                if bad and rep == 0:
                    print(f"n={n} nq={nq} k={k}: {bad[:3]}")
                    qi = int(bad[0].split()[0][1:])
                    print("   dev rows", r[qi].tolist(), "dev scores", s[qi].tolist())
                    print("   ref rows", rows[qi].tolist(), "ref scores", s64[qi].tolist())
            print(f"n={n} nq={nq} k={k}: bad counts over reps {res}", flush=True)
