#!/bin/bash
# Per-GPU shares of C3 on one GPU (r05): bench.py at the rows one rank holds
# at N = 2, 4, 8 (5M, 2.5M, 1.25M), plain (no exchange), for DESIGN.md §7's
# compute-only speed-up table. One JSON line each in gpurun_out/shares.jsonl.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for rows in 10000000 5000000 2500000 1250000; do
  timeout -k 10 300 python bench.py --rows $rows --steps 100 --warmup 10 --no-cpu-baseline --no-secondary \
    >> gpurun_out/shares.jsonl 2>> gpurun_out/shares.err || exit 1
done
