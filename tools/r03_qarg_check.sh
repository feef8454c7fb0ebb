set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VS_QUERY_ARGS_GEMV=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_qarg.log 2>&1
rc=$?; tail -2 gpurun_out/pytest_qarg.log; [ $rc -eq 0 ] || exit $rc
for a in 0 1 0 1; do export VS_QUERY_ARGS_GEMV=$a
VS_SWEEP_ROWS=2000,20000,200000 VS_SWEEP_K=10,100 timeout -k 10 300 python tools/tiny_sweep.py | tee -a gpurun_out/qarg_sweep.jsonl || exit 1
done
