#!/bin/bash
# r06 GPU batch: the speculative-bound tests (existing, cliff, writes), then
# the C3 bench (fresh batches, spec counters) at 10M and at the N = 8 share.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T="${TESTS:-tests/test_q8_spec_gpu.py tests/test_q8_spec_cliff_gpu.py tests/test_q8_spec_writes_gpu.py}"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread $T > gpurun_out/r06_spec_tests.log 2>&1 || { tail -40 gpurun_out/r06_spec_tests.log; exit 1; }
tail -8 gpurun_out/r06_spec_tests.log
if [ "${BENCH:-1}" = 1 ]; then
timeout -k 10 300 python -u bench.py --rows 1250000 --steps 100 --warmup 10 --no-cpu-baseline --no-secondary > gpurun_out/r06b_s125.json 2> gpurun_out/r06b_s125.err || exit 1
cat gpurun_out/r06b_s125.json
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/r06b_c3.json 2> gpurun_out/r06b_c3.err || exit 1
cat gpurun_out/r06b_c3.json
fi
