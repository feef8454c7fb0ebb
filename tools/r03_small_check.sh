set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_sharded_engine_gpu.py tests/test_shard_gloo.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_small.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_small.log; [ $rc -eq 0 ] || exit $rc
VS_SWEEP_ROWS=221,2000 VS_SWEEP_K=5,10,17,32,50,100 timeout -k 10 300 python tools/tiny_sweep.py | tee gpurun_out/small_sweep.jsonl || exit 1
