#!/bin/bash
# GPU-box session helper (run through gpurun). Every GPU step has its own
# time limit; a step that crashes/hangs stops the script (no retries).
#   tools/gpu_session.sh [tests] [smoke] [testsel TAG FILES.. --] [bench TAG ARGS.. --]
#                        [prof TAG ARGS.. --] [pmc TAG CTRS ARGS.. --] [tool TAG SECONDS CMD.. --]
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
stop_if_bad() {  # rc > 1 means crash / abort / timeout: start nothing more on the GPU
  if [ "$1" -gt 1 ]; then echo "STOP: step '$2' rc=$1"; exit "$1"; fi
}
while [ $# -gt 0 ]; do
  case "$1" in
    tests)
      shift
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread \
        > gpurun_out/pytest_gpu.log 2>&1
      rc=$?; echo "pytest_rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; stop_if_bad $rc pytest ;;
    testsel)  # testsel TAG PYTEST_ARGS... --
      shift; tag="$1"; shift; args=()
      while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; [ $# -gt 0 ] && shift
      timeout -k 10 900 python -u -m pytest "${args[@]}" -m gpu -x -v --timeout 600 --timeout-method thread \
        > "gpurun_out/pytest_$tag.log" 2>&1
      rc=$?; echo "pytest_${tag}_rc=$rc"; tail -3 "gpurun_out/pytest_$tag.log"; stop_if_bad $rc pytest ;;
    smoke)
      shift
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      rc=$?; echo "smoke_rc=$rc"; tail -2 gpurun_out/smoke.log; stop_if_bad $rc smoke ;;
    bench)
      shift; tag="$1"; shift; args=()
      while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; [ $# -gt 0 ] && shift
      timeout -k 10 400 python -u bench.py "${args[@]}" > "gpurun_out/bench_$tag.json" 2> "gpurun_out/bench_$tag.err"
      rc=$?; echo "bench_${tag}_rc=$rc"; cat "gpurun_out/bench_$tag.json"; stop_if_bad $rc bench ;;
    prof)
      shift; tag="$1"; shift; args=()
      while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; [ $# -gt 0 ] && shift
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_$tag" -o run \
        --output-format csv -- python bench.py "${args[@]}" > "gpurun_out/prof_$tag.log" 2>&1
      rc=$?; echo "prof_${tag}_rc=$rc"; stop_if_bad $rc prof
      cut -d, -f1-4 "gpurun_out/prof_$tag/run_kernel_stats.csv" | head -6 ;;
    pmc)
      shift; tag="$1"; shift; ctrs="$1"; shift; args=()
      while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; [ $# -gt 0 ] && shift
      timeout -s KILL 120 rocprofv3 --pmc $ctrs -d "$PWD/gpurun_out/pmc_$tag" -o run \
        --output-format csv -- python bench.py "${args[@]}" > "gpurun_out/pmc_$tag.log" 2>&1
      rc=$?; echo "pmc_${tag}_rc=$rc"; stop_if_bad $rc pmc ;;
    tool)  # tool TAG SECONDS CMD... --   (a python tool under its own limit; stdout -> gpurun_out/tool_TAG.out)
      shift; tag="$1"; shift; lim="$1"; shift; args=()
      while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done; [ $# -gt 0 ] && shift
      timeout -k 10 "$lim" python -u "${args[@]}" > "gpurun_out/tool_$tag.out" 2> "gpurun_out/tool_$tag.err"
      rc=$?; echo "tool_${tag}_rc=$rc"; tail -3 "gpurun_out/tool_$tag.out"; stop_if_bad $rc "tool $tag" ;;
    *) echo "unknown step $1"; exit 2 ;;
  esac
done
