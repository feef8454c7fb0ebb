set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/f2_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/f2_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/f2_smoke.log 2>&1 || exit 1
tail -3 gpurun_out/f2_smoke.log
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/f2_bench.json 2> gpurun_out/f2_bench.err || exit 1
cat gpurun_out/f2_bench.json
VS_SWEEP_ROWS=221,2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,50,100 timeout -k 10 300 python tools/tiny_sweep.py > gpurun_out/f2_sweep.jsonl || exit 1
cat gpurun_out/f2_sweep.jsonl
