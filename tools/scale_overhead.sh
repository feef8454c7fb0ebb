# Per-step cost of bench.py's collective path at the N=8 share (1.25M rows) on
# one GPU: plain single-rank runs against runs that force the RCCL exchange at
# world size 1 (VS_BENCH_FORCE_DIST) with the engine's communicator
# (VS_COLLECTIVE=engine: all-gather + merge on the search stream) and with
# torch.distributed's all-gather + vs_merge_keys (VS_COLLECTIVE=torch), plus a
# kernel trace of each forced form. Usage: bash tools/scale_overhead.sh
set -e
mkdir -p gpurun_out
B="--rows 1250000 --steps 400 --warmup 50 --no-cpu-baseline --no-secondary"
for i in 1 2; do
  timeout -k 10 200 python bench.py $B > gpurun_out/s125_plain_$i.json 2>gpurun_out/s125_plain_$i.err
  for c in engine torch; do
    VS_COLLECTIVE=$c VS_BENCH_FORCE_DIST=1 timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port 29511 bench.py $B > gpurun_out/s125_${c}_$i.json 2>gpurun_out/s125_${c}_$i.err
  done
done
if [ "${TRACE:-1}" = 1 ]; then
  export VS_BENCH_FORCE_DIST=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1
  R="$GRAFT_REPO_ROOT"
  cd /tmp && export TMPDIR=/tmp
  for c in engine torch; do
    export VS_COLLECTIVE=$c MASTER_PORT=$((29520 + ${#c}))
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_$c" -o run -- python3 "$R/bench.py" --rows 1250000 --steps 200 --warmup 20 --no-cpu-baseline --no-secondary > "$R/gpurun_out/s125_${c}_trace.json" 2> "$R/gpurun_out/s125_${c}_trace.err"
  done
fi
