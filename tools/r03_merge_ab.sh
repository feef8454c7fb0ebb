set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
for ts in 1 0; do
  VS_MERGE_TWO_STAGE=$ts VS_SWEEP_DTYPE=bf16 VS_SWEEP_ROWS=2000,20000,200000,5000000,12500000 VS_SWEEP_K=10,50,100 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/merge_ab.jsonl || exit 1
done
cat gpurun_out/merge_ab.jsonl
