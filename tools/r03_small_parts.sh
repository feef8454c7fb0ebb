set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
export TMPDIR=/tmp
for p in 1 2 4 16; do
  VS_SMALL_PARTS=$p timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/prof_sp$p" -o run --output-format csv -- tools/rt_floor > gpurun_out/sp$p.log 2>&1 || exit 1
  echo "parts=$p $(grep gemv_small gpurun_out/prof_sp$p/run_kernel_stats.csv | cut -d, -f2-7 | tail -c 80) $(grep vs_search gpurun_out/sp$p.log | tail -c 40)"
done
for p in 1 16; do
  VS_SMALL_PARTS=$p timeout -k 10 120 tools/rt_floor > gpurun_out/rtf_sp$p.json 2>&1 || exit 1
  echo "parts=$p $(cat gpurun_out/rtf_sp$p.json)"
done
