#!/bin/bash
# Round measurement batch on one MI355X (run through gpurun): the default
# bench line (C3) with its CPU baseline and oracle parity, the same bench
# under rocprofv3 (kernel trace + stats; the benched binary's build id in the
# file names), C1 over HTTP for both backends + the dispatch floor, and the
# concurrency-overlap trials; EXTRA="c2 c5b256 ..." adds bench configs; C3=0,
# PMC=0, C1=0, CONC=0 skip those parts (to split the batch over calls). Raw
# output stays in gpurun_out/; tools/collect_round.py copies the records into
# profiles/. Every GPU step has its own limit; the first failure stops it.
#   bash tools/measure_round.sh TAG
set -o pipefail
TAG="${1:-rNN}"
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
R="$PWD"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ "${C3:-1}" = 1 ]; then
  timeout -k 10 400 python -u bench.py > "gpurun_out/${TAG}_bench_c3.json" 2> "gpurun_out/${TAG}_bench_c3.err" || exit 1
  cat "gpurun_out/${TAG}_bench_c3.json"
  cd /tmp
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_prof_c3" -o run --output-format csv \
    -- python3 "$R/bench.py" --no-cpu-baseline > "$R/gpurun_out/${TAG}_prof_c3.json" 2> "$R/gpurun_out/${TAG}_prof_c3.err" || exit 1
  cd "$R"
fi
if [ "${PMC:-1}" = 1 ]; then
  # counters in passes of their own (no trace domains), each under a hard limit:
  # HBM bytes of the C3 main pass and the C3 single-query scan, then the MFMA
  # pipe's busy cycles and the clock of the C3 main pass
  B="--steps 10 --warmup 3 --no-cpu-baseline"
  cd /tmp
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${TAG}_pmc_fetch_c3" -o run --output-format csv \
    -- python3 "$R/bench.py" $B --no-secondary > "$R/gpurun_out/${TAG}_pmc_fetch_c3.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${TAG}_pmc_fetch_c3b1" -o run --output-format csv \
    -- python3 "$R/bench.py" $B --config c3b1 > "$R/gpurun_out/${TAG}_pmc_fetch_c3b1.log" 2>&1 || exit 1
  # (r05) the int8 pass at the N = 8 share's size (rows_per_gpu 1.25M)
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d "$R/gpurun_out/${TAG}_pmc_fetch_c3_s125" -o run --output-format csv \
    -- python3 "$R/bench.py" $B --no-secondary --rows 1250000 > "$R/gpurun_out/${TAG}_pmc_fetch_c3_s125.log" 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    -d "$R/gpurun_out/${TAG}_pmc_mfma_c3" -o run --output-format csv \
    -- python3 "$R/bench.py" $B --no-secondary > "$R/gpurun_out/${TAG}_pmc_mfma_c3.log" 2>&1 || exit 1
  cd "$R"
fi
for c in ${EXTRA:-}; do
  timeout -k 10 400 python -u bench.py --config "$c" --no-cpu-baseline > "gpurun_out/${TAG}_bench_$c.json" 2> "gpurun_out/${TAG}_bench_$c.err" || exit 1
  cat "gpurun_out/${TAG}_bench_$c.json"
done
if [ "${C1:-1}" = 1 ]; then
  timeout -k 10 300 python -u tools/c1_http.py --backend both --seconds 3 > "gpurun_out/${TAG}_c1_http.jsonl" 2> "gpurun_out/${TAG}_c1_http.err" || exit 1
  cat "gpurun_out/${TAG}_c1_http.jsonl"
  timeout -k 10 120 tools/rt_floor > "gpurun_out/${TAG}_rt_floor.json" 2> "gpurun_out/${TAG}_rt_floor.err" || exit 1
  cat "gpurun_out/${TAG}_rt_floor.json"
fi
if [ "${CONC:-1}" = 1 ]; then
  timeout -k 10 200 python -u tools/concurrency_overlap.py --out "gpurun_out/${TAG}_concurrency_overlap.json" > "gpurun_out/${TAG}_conc.out" 2>&1 || exit 1
  tail -1 "gpurun_out/${TAG}_conc.out"
fi
