#!/bin/bash
# r06: the one-query int8 tests, then C2's split and bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_q8_gemv_gpu.py > gpurun_out/r06_q8gemv_tests.log 2>&1 || { tail -30 gpurun_out/r06_q8gemv_tests.log; exit 1; }
tail -3 gpurun_out/r06_q8gemv_tests.log
bash tools/r06_c2.sh
