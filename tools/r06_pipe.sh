#!/bin/bash
# r06: share_pipe's arms (the speculative sequence priced launch by launch)
# at the N = 8 share and at 10M; one JSON line each under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
TAG="${TAG:-r06_pipe}"
timeout -k 10 150 ./tools/share_pipe 1250000 10 200 > gpurun_out/${TAG}_s125.json || exit 1
cat gpurun_out/${TAG}_s125.json
timeout -k 10 150 ./tools/share_pipe 10000000 10 40 > gpurun_out/${TAG}_10m.json || exit 1
cat gpurun_out/${TAG}_10m.json
