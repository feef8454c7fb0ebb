#!/bin/bash
# r06: the batched-path GPU tests, then environment-arm bench A/B (ARMS)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="${TESTS:-tests/test_q8_spec_gpu.py tests/test_q8_spec_writes_gpu.py tests/test_q8_gpu.py tests/test_q8_spec_cliff_gpu.py tests/test_gpu_parity.py tests/test_fp32_batched_gpu.py tests/test_configs_gpu.py}"
timeout -k 10 900 python -u -m pytest -x -q --timeout 400 --timeout-method thread $T > gpurun_out/r06_g9_tests.log 2>&1 || { tail -30 gpurun_out/r06_g9_tests.log; exit 1; }
tail -2 gpurun_out/r06_g9_tests.log
bash tools/r06_abe.sh
