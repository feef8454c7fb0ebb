set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 800 python -u -m pytest tests/test_gpu_parity.py tests/test_large_k_gpu.py tests/test_sharded_engine_gpu.py tests/test_filter_gpu.py tests/test_fp32_batched_gpu.py tests/test_service_gpu.py tests/test_configs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_one.log 2>&1
rc=$?; tail -3 gpurun_out/pytest_one.log; [ $rc -eq 0 ] || exit $rc
for one in 1 0; do
VS_GEMV_ONE=$one VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=5,10,32,100 \
    timeout -k 10 300 python tools/tiny_sweep.py >> gpurun_out/one_sweep.jsonl || exit 1
done
cat gpurun_out/one_sweep.jsonl
for c in c2 c3b1; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 10 --no-cpu-baseline > gpurun_out/bench_one_$c.json 2>gpurun_out/bench_one_$c.err || exit 1
  cat gpurun_out/bench_one_$c.json
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_one_c2" -o run --output-format csv -- python bench.py --config c2 --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/prof_one_c2.log 2>&1 || exit 1
