#!/bin/bash
# PMC passes over the int8 pass and its skeletons (tools/ablate_q8 ... ARM: one
# arm alone, REPS x 10 launches), one counter set per rocprofv3 run, each under
# its own hard limit (r05; VERDICT r04 item 2: name the cause of the MFMA
# pipe's idle cycles from counters). Every arm in ARMS runs every set.
#   ARMS="prod noepi stream mfma" ROWS=10000000 bash tools/pmc_q8.sh "CTR CTR ..." "CTR ..." ...
# Output: gpurun_out/pmcq8_<arm>_p<i>/ (csv), summarised by tools/pmc_q8_summary.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; R="$PWD"; mkdir -p gpurun_out; export TMPDIR=/tmp
for arm in ${ARMS:-prod}; do
  i=0
  for ctrs in "$@"; do
    i=$((i+1))
    cd /tmp
    timeout -s KILL 90 rocprofv3 --pmc $ctrs -d "$R/gpurun_out/pmcq8_${arm}_p$i" -o run --output-format csv \
      -- "$R/tools/ablate_q8" ${ROWS:-10000000} ${REPS:-2} 10 "$arm" > "$R/gpurun_out/pmcq8_${arm}_p$i.log" 2>&1
    rc=$?; cd "$R"; echo "$arm pass $i rc=$rc ($ctrs)"
    # 1: rocprofv3 refused a counter name (nothing ran on the GPU) -- next set;
    # anything else (limit, abort, fault) ends the script
    # (unless the program itself reported a HIP error)
    [ $rc -eq 0 ] || { [ $rc -eq 1 ] && ! grep -q "^HIP " "$R/gpurun_out/pmcq8_${arm}_p$i.log"; } || exit $rc
  done
done
