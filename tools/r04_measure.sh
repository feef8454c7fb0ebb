set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/r04_bench_c3.json 2> gpurun_out/r04_bench_c3.err || exit 1
cat gpurun_out/r04_bench_c3.json
R="$PWD"
cd /tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r04_prof_c3" -o run --output-format csv -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/r04_prof_c3.json" 2> "$R/gpurun_out/r04_prof_c3.err" || exit 1
cd "$R"
cat gpurun_out/r04_prof_c3.json
timeout -k 10 300 python -u tools/c1_http.py --backend both --seconds 3 > gpurun_out/r04_c1_http.jsonl 2> gpurun_out/r04_c1_http.err || exit 1
cat gpurun_out/r04_c1_http.jsonl
timeout -k 10 120 tools/rt_floor > gpurun_out/r04_rt_floor.json 2> gpurun_out/r04_rt_floor.err || exit 1
cat gpurun_out/r04_rt_floor.json
timeout -k 10 200 python -u tools/concurrency_overlap.py --out gpurun_out/r04_concurrency_overlap.json > gpurun_out/r04_conc.out 2>&1 || exit 1
tail -2 gpurun_out/r04_conc.out
