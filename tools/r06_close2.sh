#!/bin/bash
# r06 closing batch, part 2 (after tools/measure_round.sh r06c): C3 shares on
# one GPU, the speculative bound on / off at 10M and at the N = 8 share, the
# one-rank RCCL exchange at the share, C4's share, C5 over HTTP, and
# share_pipe's launch-by-launch arms. JSON lines under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="${TAG:-r06c}"
B="--no-cpu-baseline --no-secondary"
for rows in 5000000 2500000 1250000; do
  timeout -k 10 300 python -u bench.py --rows $rows --steps 100 --warmup 10 $B >> gpurun_out/${T}_shares.jsonl 2>> gpurun_out/${T}_shares.err || exit 1
done
tail -3 gpurun_out/${T}_shares.jsonl | cut -c1-300
for sp in 1 0; do
  VS_Q8_SPEC=$sp timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 $B >> gpurun_out/${T}_specab_10m_$sp.jsonl 2>> gpurun_out/${T}_specab.err || exit 1
  VS_Q8_SPEC=$sp timeout -k 10 300 python -u bench.py --rows 1250000 --steps 200 --warmup 10 $B >> gpurun_out/${T}_specab_s125_$sp.jsonl 2>> gpurun_out/${T}_specab.err || exit 1
done
VS_DIST_BACKEND=nccl VS_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
  --master-addr 127.0.0.1 --master-port 29533 bench.py --rows 1250000 --steps 200 --warmup 10 $B \
  > gpurun_out/${T}_s125_exchange.json 2> gpurun_out/${T}_s125_exchange.err || exit 1
tail -1 gpurun_out/${T}_s125_exchange.json | cut -c1-300
timeout -k 10 300 python -u bench.py --config c4 --rows 12500000 --steps 30 --warmup 5 $B > gpurun_out/${T}_c4share.json 2> gpurun_out/${T}_c4share.err || exit 1
cut -c1-300 gpurun_out/${T}_c4share.json
timeout -k 10 400 python -u tools/loadgen_c5.py --clients 64,256 --seconds 5 --transport both > gpurun_out/${T}_c5_loadgen.jsonl 2> gpurun_out/${T}_c5_loadgen.err || exit 1
tail -4 gpurun_out/${T}_c5_loadgen.jsonl | cut -c1-300
TAG=${T}_pipe bash tools/r06_pipe.sh > /dev/null || exit 1
echo done
