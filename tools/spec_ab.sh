#!/bin/bash
# Speculative bound A/B on one box (r05): bench.py at 10M and at the N = 8
# share with VS_Q8_SPEC=1 (default) and 0, interleaved, plus one C5 load.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
B="--steps 50 --warmup 10 --no-cpu-baseline --no-secondary"
for rep in 1 2; do
  for sp in 1 0; do
    VS_Q8_SPEC=$sp timeout -k 10 300 python bench.py $B >> gpurun_out/specab_10m_$sp.jsonl 2>> gpurun_out/specab.err || exit 1
    VS_Q8_SPEC=$sp timeout -k 10 300 python bench.py $B --rows 1250000 --steps 200 >> gpurun_out/specab_s125_$sp.jsonl 2>> gpurun_out/specab.err || exit 1
  done
done
for sp in 1 0; do
  VS_Q8_SPEC=$sp timeout -k 10 400 python -u tools/loadgen_c5.py --clients 256 --seconds 5 --transport both \
    >> gpurun_out/specab_c5_$sp.jsonl 2>> gpurun_out/specab.err || exit 1
done
