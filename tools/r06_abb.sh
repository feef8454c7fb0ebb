#!/bin/bash
# r06: bench lines (C3 main, C2, 1.25M share) and share_pipe against builds of
# the library (tools/_ab/<variant>), interleaved over two rounds, on one box.
# The in-tree library is swapped in the box's scratch copy and restored last.
#   VARS="head new" bash tools/r06_abb.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIB=$(ls -d gorilla*/lib)/libvsearch.so
cp "$LIB" /tmp/libvsearch.keep
for rep in 1 2; do
  for v in ${VARS:-head new}; do
    cp "tools/_ab/$v/libvsearch.so" "$LIB"
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 200 > gpurun_out/abb_${v}_c3_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python -u bench.py --config c2 --steps 400 --no-cpu-baseline > gpurun_out/abb_${v}_c2_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --rows 1250000 --steps 200 > gpurun_out/abb_${v}_s125_$rep.json 2>/dev/null || exit 1
    LD_LIBRARY_PATH="$PWD/tools/_ab/$v" timeout -k 10 120 ./tools/share_pipe 1250000 10 200 > gpurun_out/abb_${v}_pipe_$rep.json || exit 1
    for c in c3 c2 s125; do python3 -c "
import json;d=json.load(open('gpurun_out/abb_${v}_${c}_$rep.json'));print('$v $c $rep',d['value'],d['ms_per_step'])"; done
  done
done
cp /tmp/libvsearch.keep "$LIB"
