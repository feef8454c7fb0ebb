#!/bin/bash
# r06: C2 finish variants (tools/_ab/l<lists>p<passes>/libvsearch.so, by
# LD_LIBRARY_PATH over tools/c2_finish's runpath), interleaved over 2 rounds.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for rep in 1 2; do
  for v in ${VARS:-radix rank}; do
    LD_LIBRARY_PATH="$PWD/tools/_ab/$v" timeout -k 10 150 ./tools/c2_finish 1000000 10 200 > gpurun_out/r06_c2var_${v}_$rep.json || exit 1
    echo "$v $(cat gpurun_out/r06_c2var_${v}_$rep.json)"
  done
done
