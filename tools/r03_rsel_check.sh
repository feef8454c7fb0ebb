set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_large_k_gpu.py tests/test_service_gpu.py -m gpu -x -v --timeout 600 --timeout-method thread > gpurun_out/pytest_rsel.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_rsel.log; [ $rc -eq 0 ] || exit $rc
for f in 1 0; do
VS_RSEL_FUSED=$f VS_SWEEP_ROWS=20000,200000,10000000 VS_SWEEP_DTYPE=bf16 VS_SWEEP_K=129,1000,5000 timeout -k 10 300 python tools/tiny_sweep.py | tee -a gpurun_out/rsel_sweep.jsonl || exit 1
done
for f in 0 1; do
for rows in 10000000 200000; do
VS_RSEL_FUSED=$f VS_SWEEP_ROWS=$rows VS_SWEEP_DTYPE=bf16 VS_SWEEP_K=5000 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/rp_${f}_$rows" -o run --output-format csv -- python tools/tiny_sweep.py > gpurun_out/rp_${f}_$rows.log 2>&1 || exit 1
done
done
