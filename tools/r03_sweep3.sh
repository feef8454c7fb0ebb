set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "small_collection or gemv_single" --timeout 200 --timeout-method thread > gpurun_out/pytest_small2.log 2>&1 || { tail -5 gpurun_out/pytest_small2.log; exit 1; }
tail -1 gpurun_out/pytest_small2.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_rt2" -o run --output-format csv -- tools/rt_floor > gpurun_out/rt_floor_prof2.log 2>&1 || exit 1
grep -E "gemv_small|touch" gpurun_out/prof_rt2/run_kernel_stats.csv | cut -d, -f1-8
timeout -k 10 200 tools/rt_floor > gpurun_out/rt_floor2.json 2>&1 || exit 1
cat gpurun_out/rt_floor2.json
timeout -k 10 200 python -u tools/c1_http.py --backend gpu > gpurun_out/c1_hoist.jsonl 2>/dev/null || exit 1
cat gpurun_out/c1_hoist.jsonl
echo done
