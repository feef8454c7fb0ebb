#!/bin/bash
# Select A/B on one box (r05): share_pipe against several builds of the
# library (tools/_ab/<variant>/libvsearch.so, picked by LD_LIBRARY_PATH over
# the binary's runpath), interleaved over two rounds, at the N = 8 share,
# at 10M and at one C5 collection. Outputs gpurun_out/ab_<variant>_<cfg>_<rep>.json.
#   bash tools/select_ab.sh VARIANT...
set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@"; do
    L="$PWD/tools/_ab/$v"
    LD_LIBRARY_PATH="$L" timeout -k 10 120 ./tools/share_pipe 1250000 10 200 > gpurun_out/ab_${v}_s125_$rep.json || exit 1
    LD_LIBRARY_PATH="$L" timeout -k 10 120 ./tools/share_pipe 10000000 10 40 > gpurun_out/ab_${v}_10m_$rep.json || exit 1
    LD_LIBRARY_PATH="$L" timeout -k 10 120 ./tools/share_pipe 5000000 50 40 1024 > gpurun_out/ab_${v}_c5_$rep.json || exit 1
  done
done
