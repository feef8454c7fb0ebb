set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_full.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_full.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit 1
tail -3 gpurun_out/smoke.log
VS_SWEEP_ROWS=221,2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,50,100 \
    timeout -k 10 300 python tools/tiny_sweep.py > gpurun_out/final_sweep.jsonl || exit 1
VS_SWEEP_DTYPE=bf16 VS_SWEEP_ROWS=2000,20000,200000,5000000,12500000 VS_SWEEP_K=10,50,100 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/final_sweep.jsonl || exit 1
cat gpurun_out/final_sweep.jsonl
for c in c2 c3b1; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_fin_$c.json 2>gpurun_out/bench_fin_$c.err || exit 1
  cat gpurun_out/bench_fin_$c.json
done
timeout -k 10 200 python tools/c1_http.py --backend gpu --seconds 3 > gpurun_out/c1_http.jsonl 2>gpurun_out/c1_http.err || exit 1
cat gpurun_out/c1_http.jsonl
