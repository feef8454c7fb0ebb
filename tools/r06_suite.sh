#!/bin/bash
# r06: the full -m gpu suite (no -x: every failure reported) and smoke().
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG="${TAG:-r06_suite}"
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}.log 2>&1
rc=$?; echo "pytest_rc=$rc"; grep -E "FAILED|ERROR" gpurun_out/${TAG}.log | head -20; tail -2 gpurun_out/${TAG}.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.log
