#!/bin/bash
# r06: C2's single-query step split (tools/c2_finish) and the C2 bench line.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
TAG="${TAG:-r06_c2}"
timeout -k 10 150 ./tools/c2_finish 1000000 10 200 > gpurun_out/${TAG}_finish.json || exit 1
cat gpurun_out/${TAG}_finish.json
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 300 python -u bench.py --config c2 --steps 200 --no-cpu-baseline > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err || exit 1
cat gpurun_out/${TAG}_bench.json
fi
