#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_q8_gemv_gpu.py tests/test_q8_spec_gpu.py > gpurun_out/r06_g5_tests.log 2>&1 || { tail -40 gpurun_out/r06_g5_tests.log; exit 1; }
tail -3 gpurun_out/r06_g5_tests.log
timeout -k 10 300 python -u bench.py --config c2 --steps 200 --no-cpu-baseline > gpurun_out/r06_g5_c2.json 2> gpurun_out/r06_g5_c2.err || exit 1
cut -c1-300 gpurun_out/r06_g5_c2.json
