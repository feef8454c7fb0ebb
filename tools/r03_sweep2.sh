set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
timeout -k 10 600 python -u -m pytest tests/test_large_k_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_lk3.log 2>&1
rc=$?; echo "pytest_rc=$rc"; tail -2 gpurun_out/pytest_lk3.log; [ $rc -ne 0 ] && exit 1
timeout -k 10 200 python -u tools/large_k_bench.py --ks 10,128,129,1024,5000 --reps 15 > gpurun_out/lk3.jsonl 2>/dev/null || exit 1
cat gpurun_out/lk3.jsonl
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_rt" -o run --output-format csv -- tools/rt_floor > gpurun_out/rt_floor_prof.log 2>&1 || exit 1
cut -d, -f1-8 gpurun_out/prof_rt/run_kernel_stats.csv | head -8
echo done
