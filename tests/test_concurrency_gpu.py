"""Concurrent host-API calls on one single-device engine (vs_search waits for
the device outside the engine's work lock since r02, vs_engine.cpp
search_host): searches of mixed batch sizes and k from several threads,
while another thread upserts into a second collection (growing its capacity)
and a third creates / drops collections. Every concurrent answer must equal
the same search run alone afterwards, bit for bit (the engine is
deterministic), and a sample of them the oracle."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_concurrent_searches_with_upserts(pkg, orc):
    n, dim = 50_000, 768
    eng = pkg.VectorEngine(device=0)
    try:
        eng.create_collection("a", dim, pkg.METRIC_COSINE, pkg.DTYPE_BF16)
        eng.generate("a", n, 777)
        eng.create_collection("b", dim, pkg.METRIC_COSINE, pkg.DTYPE_F32)
        rng = np.random.default_rng(3)
        plans = []  # (thread, i) -> (nq, k, query seed row)
        for t in range(4):
            for i in range(12):
                nq = int(rng.choice([1, 2, 7, 64, 256, 300]))
                k = int(rng.choice([1, 10, 50, 100, 200]))
                plans.append((t, i, nq, k, int(rng.integers(0, 10_000))))
        results = {}
        errors = []
        stop = threading.Event()

        def searcher(t):
            try:
                for (tt, i, nq, k, q0) in plans:
                    if tt != t:
                        continue
                    Q = orc.generate(orc.SEED_QUERY, q0, nq, dim)
                    results[(t, i)] = eng.search("a", Q, k)
            except Exception as e:  # noqa: BLE001
                errors.append(("search", t, repr(e)))

        def upserter():
            try:
                r = 0
                while not stop.is_set():
                    m = 3000
                    V = orc.generate(91, r, m, dim)
                    eng.upsert("b", list(range(r, r + m)), V)
                    r += m
            except Exception as e:  # noqa: BLE001
                errors.append(("upsert", repr(e)))

        def churner():
            try:
                j = 0
                while not stop.is_set():
                    name = f"tmp{j % 3}"
                    eng.create_collection(name, 128, pkg.METRIC_DOT, pkg.DTYPE_F32)
                    eng.generate(name, 1000, j)
                    eng.search(name, orc.generate(5, j, 3, 128), 5)
                    eng.drop_collection(name)
                    j += 1
            except Exception as e:  # noqa: BLE001
                errors.append(("churn", repr(e)))

        th = [threading.Thread(target=searcher, args=(t,)) for t in range(4)]
        bg = [threading.Thread(target=upserter), threading.Thread(target=churner)]
        for x in bg + th:
            x.start()
        for x in th:
            x.join()
        stop.set()
        for x in bg:
            x.join()
        assert not errors, errors[:3]
        X = orc.generate(777, 0, n, dim, bf16=True)
        checked = 0
        for (t, i, nq, k, q0) in plans:
            Q = orc.generate(orc.SEED_QUERY, q0, nq, dim)
            s1, r1, c1 = results[(t, i)]
            s2, r2, c2 = eng.search("a", Q, k)
            assert np.array_equal(r1, r2) and np.array_equal(c1, c2), (t, i, nq, k)
            assert np.array_equal(s1.view(np.uint32), s2.view(np.uint32)), (t, i, nq, k)
            if checked < 6 and nq <= 7:
                Qp = orc.preprocess(Q, True, True)
                s32, s64, rr, cc = orc.search(X, Qp, k)
                bad = orc.check_topk(s1, r1, c1, s64, rr, cc, orc.rescore(X, Qp, r1, c1), 1e-5)
                assert not bad, bad[:3]
                checked += 1
        assert checked > 0
    finally:
        eng.close()
