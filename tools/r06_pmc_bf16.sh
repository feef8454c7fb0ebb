#!/bin/bash
# r06: counters of the bf16 MFMA pass (the C3 batch with
# the int8 copy off, VS_Q8=0) in one --pmc pass of its own: GRBM_GUI_ACTIVE,
# SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, SQ_WAVE_CYCLES; and its kernel
# trace (durations) in a second run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; R=$PWD; mkdir -p gpurun_out; export TMPDIR=/tmp
TAG="${TAG:-r06_bf16}"
cd /tmp
VS_Q8=0 timeout -s KILL 150 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
  -d "$R/gpurun_out/${TAG}_pmc_mfma" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > "$R/gpurun_out/${TAG}_pmc_mfma.log" 2>&1 || exit 1
VS_Q8=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$R/gpurun_out/${TAG}_trace" -o run --output-format csv \
  -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu-baseline --no-secondary > "$R/gpurun_out/${TAG}_trace.log" 2>&1 || exit 1
cd "$R"
tail -1 gpurun_out/${TAG}_trace.log
