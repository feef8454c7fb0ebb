#!/bin/bash
# r06: full -m gpu suite + smoke (TAG), then C2, C3 and the 1.25M share lines
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG="${TAG:-r06_g7}"
bash tools/r06_suite.sh || exit 1
timeout -k 10 300 python -u bench.py --config c2 --steps 200 --no-cpu-baseline > gpurun_out/${TAG}_c2.json 2> gpurun_out/${TAG}_c2.err || exit 1
timeout -k 10 400 python -u bench.py --no-cpu-baseline > gpurun_out/${TAG}_c3.json 2> gpurun_out/${TAG}_c3.err || exit 1
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-secondary --rows 1250000 --steps 200 > gpurun_out/${TAG}_s125.json 2> gpurun_out/${TAG}_s125.err || exit 1
for f in c2 c3 s125; do python3 -c "
import json,sys;d=json.load(open('gpurun_out/${TAG}_$f.json'));print('$f',d['value'],d['ms_per_step'],d['roofline']['frac'],d.get('spec_fallbacks'),(d.get('secondary') or {}).get('value'))"; done
