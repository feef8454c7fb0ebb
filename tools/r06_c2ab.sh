#!/bin/bash
# r06: C2 finish A/B (the last merge: list walk vs tournament), interleaved.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for rep in 1 2; do
  for t in 0 1; do
    VS_Q8G_TOURNEY=$t timeout -k 10 150 ./tools/c2_finish 1000000 10 200 > gpurun_out/r06_c2ab_t${t}_$rep.json || exit 1
    cat gpurun_out/r06_c2ab_t${t}_$rep.json
  done
done
VS_Q8G_TOURNEY=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_q8_gemv_gpu.py > gpurun_out/r06_c2ab_tests.log 2>&1 || { tail -30 gpurun_out/r06_c2ab_tests.log; exit 1; }
tail -2 gpurun_out/r06_c2ab_tests.log
