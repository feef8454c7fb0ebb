"""Cross-shard merge cost (vs_merge_keys) at the bench's N-GPU shapes.

    python tools/merge_bench.py [LIB]  # run under rocprofv3 --kernel-trace --stats

For P in (2, 4, 8): P per-shard top-10 lists of 256 queries (random unique
keys) merged into the global top-10, 200 times; then 768 lists (the GEMV
single-query merge). Each shape is checked once against a host sort.
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    if len(sys.argv) > 1:  # another build of libvsearch.so (A/B)
        pkg.load_library(sys.argv[1])
    eng = pkg.VectorEngine(device=0)
    k = 10
    rng = np.random.default_rng(0)
    # (lists, queries): cross-shard merges at the bench's N, then the
    # single-query GEMV merge (768 workgroup lists)
    for P, nq in ((2, 256), (4, 256), (8, 256), (768, 1), (768, 4)):
        keys = rng.choice(2**62, size=(P, nq, k), replace=False).astype(np.uint64)
        keys = -np.sort(-keys.view(np.int64), axis=2).view(np.uint64)  # each list descending
        d_in = torch.from_numpy(keys.view(np.int64)).cuda()
        d_out = torch.zeros((nq, k), dtype=torch.int64, device="cuda")
        for _ in range(200):
            eng.merge_keys(d_in.data_ptr(), P, nq, k, k, d_out.data_ptr())
        torch.cuda.synchronize()
        got = d_out.cpu().numpy().view(np.uint64)
        exp = -np.sort(-keys.transpose(1, 0, 2).reshape(nq, P * k).view(np.int64), axis=1)[:, :k]
        assert np.array_equal(got, exp.view(np.uint64)), P
        print(f"P={P} nq={nq}: ok", flush=True)
    eng.close()


if __name__ == "__main__":
    main()
