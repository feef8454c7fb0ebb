#!/bin/bash
# select A/B batch (r05): the int8 GPU tests, then share_pipe at the N = 8
# share and at 10M (stage clocks and counts), TAG names the outputs.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
TAG="${1:-sel}"
bash tools/gpu_session.sh testsel q8 tests/test_q8_gpu.py tests/test_filter_gpu.py tests/test_gpu_parity.py -- || exit 1
timeout -k 10 120 ./tools/share_pipe 1250000 10 200 > gpurun_out/${TAG}_s125.json || exit 1
timeout -k 10 120 ./tools/share_pipe 10000000 10 40 > gpurun_out/${TAG}_10m.json || exit 1
timeout -k 10 120 ./tools/share_pipe 5000000 50 40 1024 > gpurun_out/${TAG}_c5.json || exit 1
