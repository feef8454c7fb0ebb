#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
TESTS="tests/test_q8_spec_gpu.py tests/test_q8_spec_cliff_gpu.py tests/test_q8_spec_writes_gpu.py tests/test_q8_gpu.py" BENCH=1 bash tools/r06_g2.sh || exit 1
TAG=r06d_pipe bash tools/r06_pipe.sh | cut -c1-400
