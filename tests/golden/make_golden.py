"""Generates the committed golden fixtures of tests/golden/ from the oracle.

The reference holds no fixtures for this path, so these are
oracle outputs frozen at commit time: they pin the oracle (and through it the
device path) against regressions, and they fix the synthetic generator by a
digest so the GPU box can regenerate identical corpora without shipping data.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import oracle  # noqa: E402

N, DIM, NQ = 4096, 768, 32
KS = (1, 5, 10, 100)


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def main():
    out = {}
    X32 = oracle.generate(oracle.SEED_CORPUS, 0, N, DIM, bf16=False)
    Xb = oracle.generate_raw(oracle.SEED_CORPUS, 0, N, DIM, bf16=True)
    Q = oracle.generate(oracle.SEED_QUERY, 0, NQ, DIM, bf16=False)
    out["corpus_f32_sha256"] = digest(X32)
    out["corpus_bf16_sha256"] = digest(Xb)
    out["queries_f32_sha256"] = digest(Q)
    np.savez_compressed(os.path.join(HERE, "gen_head.npz"), corpus_f32=X32[:8],
                        corpus_bf16_bits=Xb[:8], queries_f32=Q[:4],
                        ints_row0=oracle.np_gen_ints(oracle.SEED_CORPUS, 0, 1, DIM)[0])
    arrays = {}
    for tag, bf16 in (("f32", False), ("bf16", True)):
        X = oracle.generate(oracle.SEED_CORPUS, 0, N, DIM, bf16=bf16)
        Qp = oracle.preprocess(Q, cosine=True, bf16=bf16)
        arrays[f"qpre_{tag}"] = Qp
        for k in KS:
            s32, s64, rows, cnt = oracle.search(X, Qp, k)
            arrays[f"rows_{tag}_k{k}"] = rows
            arrays[f"scores64_{tag}_k{k}"] = s64
    np.savez_compressed(os.path.join(HERE, "search_4096x768.npz"), **arrays)
    # preprocess edge cases (raw inputs and the oracle's stored values)
    rng = np.random.default_rng(7)
    edge = np.stack([
        np.zeros(DIM, np.float32),
        np.full(DIM, 1e-30, np.float32),
        Q[0],                                   # already unit: kept bit-exactly
        (Q[1] * 3.5).astype(np.float32),
        rng.standard_normal(DIM).astype(np.float32) * 1e3,
        np.eye(1, DIM, 5, dtype=np.float32)[0] * -2.0,
    ])
    np.savez_compressed(os.path.join(HERE, "preprocess_edge.npz"), raw=edge,
                        cosine_f32=oracle.preprocess(edge, True, False),
                        cosine_bf16=oracle.preprocess(edge, True, True),
                        dot_f32=oracle.preprocess(edge, False, False))
    with open(os.path.join(HERE, "digests.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
