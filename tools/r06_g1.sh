set -o pipefail
cd "${GRAFT_REPO_ROOT}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 tools/launch_floor > gpurun_out/r06_launch_floor.json 2>&1 || exit 1
cat gpurun_out/r06_launch_floor.json
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 100 --warmup 10 --no-cpu-baseline --no-secondary > gpurun_out/r06a_s125.json 2> gpurun_out/r06a_s125.err || exit 1
cat gpurun_out/r06a_s125.json
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/r06a_prof_s125" -o run --output-format csv -- python3 "$R/bench.py" --rows 1250000 --steps 100 --warmup 10 --no-cpu-baseline --no-secondary > "$R/gpurun_out/r06a_prof_s125.json" 2> "$R/gpurun_out/r06a_prof_s125.err" || exit 1
echo done
