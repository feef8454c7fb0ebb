#!/bin/bash
# GPU-box PMC session over the ablation binary: one counter pass per run.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$PWD/gpurun_out/pmc_p$i" -o run --output-format csv -- ./tools/ablate_mfma ${ROWS:-10000000} ${REPS:-2} > gpurun_out/pmc_p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
