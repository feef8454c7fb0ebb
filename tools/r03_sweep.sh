# r03 GPU session: large-k correctness + timing, contexts on C5 / C1
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 900 python -u -m pytest tests/test_large_k_gpu.py tests/test_gpu_parity.py tests/test_filter_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lk2.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -2 gpurun_out/pytest_lk2.log; [ $rc -gt 1 ] && exit $rc
timeout -k 10 200 python -u tools/large_k_bench.py --ks 10,128,129,256,1024,5000,500000 --reps 15 > gpurun_out/lk2.jsonl 2>/dev/null || exit 1
cat gpurun_out/lk2.jsonl
timeout -k 10 300 python -u tools/loadgen_c5.py --transport both --clients 16,64,256 --seconds 4 --unbatched-clients 0 > gpurun_out/c5_heavy.jsonl 2>/dev/null || exit 1
cat gpurun_out/c5_heavy.jsonl

timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "small_collection" --timeout 200 --timeout-method thread > gpurun_out/pytest_small.log 2>&1 || { tail -5 gpurun_out/pytest_small.log; exit 1; }
tail -1 gpurun_out/pytest_small.log
timeout -k 10 200 tools/rt_floor > gpurun_out/rt_floor.json 2>&1 || exit 1
cat gpurun_out/rt_floor.json
timeout -k 10 200 python -u tools/c1_http.py --backend gpu > gpurun_out/c1_multiwg.jsonl 2>/dev/null || exit 1
cat gpurun_out/c1_multiwg.jsonl
echo done
