#!/bin/bash
# r06h: library A/B (tools/_ab/<variant>/libvsearch.so swapped into the
# box's scratch copy, restored last): the 1.25M share with speculation on
# and off, C3, and share_pipe's select stage clocks, interleaved over REPS
# rounds on one box. One line per run on stdout.
#   VARS="head new" REPS=3 bash tools/r06_abh.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LIB=$(ls -d gorilla*/lib)/libvsearch.so
cp "$LIB" /tmp/libvsearch.keep
B="--no-cpu-baseline --no-secondary"
for rep in $(seq 1 ${REPS:-3}); do
  for v in ${VARS:-head new}; do
    cp "tools/_ab/$v/libvsearch.so" "$LIB"
    timeout -k 10 200 python -u bench.py $B --rows 1250000 --steps 200 > gpurun_out/abh_${v}_s125_$rep.json 2>/dev/null || exit 1
    VS_Q8_SPEC=0 timeout -k 10 200 python -u bench.py $B --rows 1250000 --steps 200 > gpurun_out/abh_${v}_s125off_$rep.json 2>/dev/null || exit 1
    timeout -k 10 200 python -u bench.py $B --steps 50 > gpurun_out/abh_${v}_c3_$rep.json 2>/dev/null || exit 1
    LD_LIBRARY_PATH="$PWD/tools/_ab/$v" timeout -k 10 120 ./tools/share_pipe 1250000 10 200 > gpurun_out/abh_${v}_pipe_$rep.json || exit 1
    for c in s125 s125off c3; do python3 -c "
import json;d=json.load(open('gpurun_out/abh_${v}_${c}_$rep.json'));print('$v $c $rep',d['value'],d['ms_per_step'])"; done
    python3 -c "
import json;d=json.load(open('gpurun_out/abh_${v}_pipe_$rep.json'));print('$v pipe $rep', d['specseq_fb_us'], d['full_us'], d['sel_p1_us_med']-d['sel_survivors_us_med'], d['sel_end_us_med'], d['sel_end_us_max'])"
  done
done
cp /tmp/libvsearch.keep "$LIB"
