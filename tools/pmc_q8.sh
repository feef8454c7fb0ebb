#!/bin/bash
# PMC passes over the int8 pass alone (tools/ablate_q8 ... prod: the product
# kernel, REPS x 10 launches at 10M rows), one counter set per rocprofv3 run,
# each under its own hard limit (r05; VERDICT r04 item 2: name the cause of
# the MFMA pipe's idle cycles from counters). Summaries: tools/pmc_summary.py.
#   bash tools/pmc_q8.sh "CTR CTR ..." "CTR ..." ...
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; R="$PWD"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for ctrs in "$@"; do
  i=$((i+1))
  cd /tmp
  timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/pmcq8_p$i" -o run --output-format csv \
    -- "$R/tools/ablate_q8" ${ROWS:-10000000} ${REPS:-2} 10 prod > "$R/gpurun_out/pmcq8_p$i.log" 2>&1
  rc=$?; cd "$R"; echo "pass $i rc=$rc ($ctrs)"; [ $rc -eq 0 ] || exit $rc
done
