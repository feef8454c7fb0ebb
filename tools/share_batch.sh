#!/bin/bash
# r05 share batch (run through gpurun): the int8/parity GPU tests, share_pipe
# at the N = 8 share and at 10M with and without the select's quarter bound,
# bench.py at 1.25M rows plain and with the RCCL exchange forced at one rank,
# and a FETCH_SIZE pass of the share's int8 pass. Every GPU step under its own
# limit; the first failure stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; R="$PWD"; mkdir -p gpurun_out; export TMPDIR=/tmp
bash tools/gpu_session.sh testsel q8 tests/test_q8_gpu.py tests/test_gpu_parity.py -- || exit 1
for p0 in 1 0; do
  VS_Q8_SEL_P0=$p0 timeout -k 10 120 ./tools/share_pipe 1250000 10 200 > gpurun_out/spp_s125_$p0.json || exit 1
  VS_Q8_SEL_P0=$p0 timeout -k 10 120 ./tools/share_pipe 10000000 10 40 > gpurun_out/spp_10m_$p0.json || exit 1
done
B="--rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary"
timeout -k 10 300 python bench.py $B > gpurun_out/xs_share_plain.json 2> gpurun_out/xs_share_plain.err || exit 1
env VS_DIST_BACKEND=nccl VS_BENCH_FORCE_DIST=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node=1 --master-addr 127.0.0.1 --master-port $((29500 + RANDOM % 1000)) bench.py $B \
  > gpurun_out/xs_share_dist.json 2> gpurun_out/xs_share_dist.err || exit 1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/xs_pmc_s125" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --rows 1250000 \
  > "$R/gpurun_out/xs_pmc_s125.log" 2>&1 || exit 1
