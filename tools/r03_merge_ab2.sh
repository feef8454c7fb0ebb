set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 1 0; do
  VS_MERGE_TOURNEY=$t VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=5,10,32 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/merge_ab2.jsonl || exit 1
  VS_MERGE_TOURNEY=$t VS_SWEEP_ROWS=1000000 VS_SWEEP_K=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$PWD/gpurun_out/pm_t$t" -o run --output-format csv -- python tools/tiny_sweep.py > gpurun_out/pm_t$t.log 2>&1 || exit 1
done
cat gpurun_out/merge_ab2.jsonl
