set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for one in 2 1 0; do
VS_GEMV_ONE=$one VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,100 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/one_sweep.jsonl || exit 1
for rows in 20000 200000; do
VS_GEMV_ONE=$one VS_SWEEP_ROWS=$rows VS_SWEEP_K=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/pm_one_${one}_$rows" -o run --output-format csv -- python tools/tiny_sweep.py > gpurun_out/pm_one_${one}_$rows.log 2>&1 || exit 1
done
done
cat gpurun_out/one_sweep.jsonl
