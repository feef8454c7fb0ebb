#!/bin/bash
# Per-step cost of bench.py's exchange at one shard's size on one GPU (r05):
# the N = 8 share (1.25M rows) plain, and with the RCCL all-gather + merge
# forced at world size 1 (VS_BENCH_FORCE_DIST=1, nccl, the engine's
# communicator) on the search stream (VS_EXCHANGE_OVERLAP=0) and on a stream
# of its own (VS_EXCHANGE_OVERLAP=1, off by default since r05: batch i's exchange overlaps batch i + 1's search).
# Each arm twice, interleaved. One JSON line per run in gpurun_out/xo_<arm>.jsonl.
#   bash tools/exchange_overlap.sh [ROWS]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
ROWS="${1:-1250000}"
B="--rows $ROWS --steps 200 --warmup 20 --no-cpu-baseline --no-secondary"
run_dist() {  # $1 arm, $2 overlap
  env VS_DIST_BACKEND=nccl VS_BENCH_FORCE_DIST=1 VS_EXCHANGE_OVERLAP="$2" MASTER_ADDR=127.0.0.1 \
    timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
    --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py $B \
    >> "gpurun_out/xo_$1.jsonl" 2>> "gpurun_out/xo_$1.err"
}
for rep in 1 2; do
  timeout -k 10 300 python bench.py $B >> gpurun_out/xo_plain.jsonl 2>> gpurun_out/xo_plain.err || exit 1
  run_dist sync 0 || exit 1
  run_dist overlap 1 || exit 1
done
for a in plain sync overlap; do
  python - "$a" <<'EOF'
import json, sys
a = sys.argv[1]
for l in open(f"gpurun_out/xo_{a}.jsonl"):
    if l.startswith("{"):
        d = json.loads(l)
        print(a, d["ms_per_step"], d["value"], d["config"].get("exchange_overlapped"), d["roofline"]["kernel_ms"])
EOF
done
