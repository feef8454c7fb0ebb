#!/bin/bash
# r05 closing batch (run through gpurun): C5 closed-loop load at 64 / 256
# clients over both transports, twice; the N = 8 share's bench line plain
# and with the one-rank RCCL exchange; C4's share (12.5M rows, k = 100).
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for rep in 1 2; do
  timeout -k 10 400 python -u tools/loadgen_c5.py --clients 64,256 --seconds 5 --transport both \
    >> gpurun_out/fin_c5.jsonl 2>> gpurun_out/fin_c5.err || exit 1
done
B="--rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary"
timeout -k 10 300 python bench.py $B > gpurun_out/fin_share.json 2> gpurun_out/fin_share.err || exit 1
env VS_DIST_BACKEND=nccl VS_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node=1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py $B \
  > gpurun_out/fin_share_rccl1.json 2> gpurun_out/fin_share_rccl1.err || exit 1
timeout -k 10 400 python bench.py --config c4 --rows 12500000 --steps 30 --warmup 5 --no-cpu-baseline \
  > gpurun_out/fin_c4share.json 2> gpurun_out/fin_c4share.err || exit 1
