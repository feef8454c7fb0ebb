#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
bash tools/r06_c2var.sh || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_q8_gemv_gpu.py > gpurun_out/r06_g6_tests.log 2>&1 || { tail -40 gpurun_out/r06_g6_tests.log; exit 1; }
tail -2 gpurun_out/r06_g6_tests.log
