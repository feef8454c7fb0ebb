"""One-query merge latency by shape (vs_merge_keys, nq = 1), for rocprofv3.

    rocprofv3 --kernel-trace -d DIR -o run --output-format csv -- python tools/merge_lat.py
    python tools/merge_lat.py --parse DIR/run_kernel_trace.csv

For each (lists, k): REPS merges of sorted random lists of k distinct keys
(the single-query GEMV merge's input: one list per scan workgroup), checked
once against a host sort. --parse groups merge_keys_kernel durations by
shape, in launch order, and prints one JSON line.
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
SHAPES = [(64, 10), (256, 10), (768, 5), (768, 10), (768, 32), (768, 100), (125, 10), (625, 10)]
REPS = 300


def parse(path):
    import csv
    d = [int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
         for r in csv.DictReader(open(path)) if "merge_keys_kernel" in r["Kernel_Name"]]
    out = {}
    for i, (L, k) in enumerate(SHAPES):
        seg = np.array(d[i * (REPS + 1) + 1:(i + 1) * (REPS + 1)]) / 1e3
        out[f"L{L}_k{k}"] = {"median_us": round(float(np.median(seg)), 2),
                             "min_us": round(float(seg.min()), 2)}
    print(json.dumps({"tool": "merge_lat", "kernel_us": out}))


def main():
    import torch
    import __graft_entry__ as ge
    pkg = ge.load_package()
    eng = pkg.VectorEngine(device=0)
    rng = np.random.default_rng(3)
    st = torch.cuda.current_stream().cuda_stream
    for L, k in SHAPES:
        keys = np.sort(rng.choice(2**62, size=(L, k), replace=False).astype(np.uint64) + 1,
                       axis=1)[:, ::-1].copy()
        d = torch.from_numpy(keys.view(np.int64)).cuda()
        out = torch.zeros((1, k), dtype=torch.int64, device="cuda")
        for _ in range(REPS + 1):  # the first launch is the check
            eng.merge_keys(d.data_ptr(), L, 1, k, k, out.data_ptr(), st)
            if _ == 0:
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint64)[0]
                want = np.sort(keys.ravel())[::-1][:k]
                assert np.array_equal(got, want), (L, k)
        torch.cuda.synchronize()
    eng.close()
    print("ok")


if __name__ == "__main__":
    if len(sys.argv) > 2 and sys.argv[1] == "--parse":
        parse(sys.argv[2])
    else:
        main()
