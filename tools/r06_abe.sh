#!/bin/bash
# r06: bench lines (C3 main, C2, 1.25M share) under environment arms of the
# in-tree build, interleaved over two rounds on one box.
#   ARMS="off:VS_Q8_SEL_VERIFY=0 on:VS_Q8_SEL_VERIFY=1" bash tools/r06_abe.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for rep in 1 2; do
  for arm in $ARMS; do
    v=${arm%%:*}; e=${arm#*:}
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --steps 200 > gpurun_out/abe_${v}_c3_$rep.json 2>/dev/null || exit 1
    env $e timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --rows 1250000 --steps 200 > gpurun_out/abe_${v}_s125_$rep.json 2>/dev/null || exit 1
    for c in c3 s125; do python3 -c "
import json;d=json.load(open('gpurun_out/abe_${v}_${c}_$rep.json'));print('$v $c $rep',d['value'],d['ms_per_step'],d['spec_stats'])"; done
  done
done
