set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_large_k_gpu.py tests/test_sharded_engine_gpu.py tests/test_filter_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_merge.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_merge.log; [ $rc -eq 0 ] || exit $rc
export VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=10,32,50,100,128
timeout -k 10 200 python tools/tiny_sweep.py > gpurun_out/sweep_merge.jsonl || exit 1
cat gpurun_out/sweep_merge.jsonl
VS_SWEEP_ROWS=200000 VS_SWEEP_K=100 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$PWD/gpurun_out/pm_merge" -o run --output-format csv -- python tools/tiny_sweep.py > gpurun_out/pm_merge.log 2>&1 || exit 1
