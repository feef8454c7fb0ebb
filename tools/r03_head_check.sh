set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h_smoke.log 2>&1 || exit 1
tail -3 gpurun_out/h_smoke.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_http_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/h_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/h_pytest.log; [ $rc -eq 0 ] || exit $rc
VS_SWEEP_ROWS=221,2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,50,100 timeout -k 10 300 python tools/tiny_sweep.py | tee gpurun_out/h_sweep.jsonl || exit 1
timeout -k 10 200 python tools/c1_http.py --backend gpu --seconds 3 | tee gpurun_out/h_c1.jsonl || exit 1
