set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 1 0; do
VS_MERGE_TOURNEY=$t timeout -k 10 120 rocprofv3 --kernel-trace -d "$PWD/gpurun_out/ml_$t" -o run --output-format csv -- python tools/merge_lat.py > gpurun_out/ml_$t.log 2>&1 || { tail -5 gpurun_out/ml_$t.log; exit 1; }
python tools/merge_lat.py --parse gpurun_out/ml_$t/run_kernel_trace.csv | tee -a gpurun_out/merge_lat.jsonl
done
