set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_large_k_gpu.py tests/test_sharded_engine_gpu.py tests/test_filter_gpu.py tests/test_fp32_batched_gpu.py tests/test_service_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_merge3.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_merge3.log; [ $rc -eq 0 ] || exit $rc
for t in 1 0; do
  VS_MERGE_TOURNEY=$t VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,50,100 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/merge_ab3.jsonl || exit 1
  VS_MERGE_TOURNEY=$t VS_SWEEP_ROWS=1000000 VS_SWEEP_K=10 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$PWD/gpurun_out/pm3_t$t" -o run --output-format csv -- python tools/tiny_sweep.py > gpurun_out/pm3_t$t.log 2>&1 || exit 1
done
VS_DIRECT_COMPLETION=0 VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,50,100 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/merge_ab3.jsonl || exit 1
cat gpurun_out/merge_ab3.jsonl
