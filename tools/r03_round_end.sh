# Round-end measurement batch on one MI355X: GPU tests, smoke, the default
# bench line (C3) with its CPU baseline, its rocprofv3 kernel trace, the other
# bench configs and C5 through the server process. Each GPU step has its own
# limit; the first failure stops the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/re_pytest.log 2>&1
rc=$?; tail -2 gpurun_out/re_pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/re_smoke.log 2>&1 || exit 1
tail -3 gpurun_out/re_smoke.log
timeout -k 10 400 python -u bench.py > gpurun_out/re_bench_c3.json 2> gpurun_out/re_bench_c3.err || exit 1
cat gpurun_out/re_bench_c3.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/re_prof_c3" -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/re_prof_c3.log 2>&1 || exit 1
for c in c2 c2b256 c5b256 c4b1; do
  timeout -k 10 400 python -u bench.py --config $c --no-cpu-baseline > gpurun_out/re_bench_$c.json 2> gpurun_out/re_bench_$c.err || exit 1
  cat gpurun_out/re_bench_$c.json
done
timeout -k 10 400 python -u tools/loadgen_c5.py --server --transport http --clients 64,256 --seconds 5 > gpurun_out/re_c5_server.jsonl 2> gpurun_out/re_c5_server.err || exit 1
cat gpurun_out/re_c5_server.jsonl
