#!/bin/bash
# GPU-box ablation session: parity tests first, then the ablation binary.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
if [ "${1:-}" = "tests" ]; then
  timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
  rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
timeout -k 10 180 ./tools/ablate_mfma ${ROWS:-10000000} ${REPS:-8} > gpurun_out/abl.txt 2>&1; rc=$?
cat gpurun_out/abl.txt; exit $rc
