# rocprof kernel stats of single-query searches on mid-size collections
# (list path vs large-k path), one size / k per run so the stats separate
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for cfg in "200000 10 129" "200000 100 129" "200000 100 33" "20000 100 129" "20000 10 129"; do
  set -- $cfg
  tag="r${1}_k${2}_lk${3}"
  VS_SWEEP_ROWS=$1 VS_SWEEP_K=$2 VS_LARGE_K_FROM=$3 timeout -k 10 120 rocprofv3 --kernel-trace --stats \
    -d "$PWD/gpurun_out/pm_$tag" -o run --output-format csv -- python tools/tiny_sweep.py \
    > "gpurun_out/pm_$tag.log" 2>&1 || { echo "FAIL $tag"; exit 1; }
  echo "== $tag"; tail -1 "gpurun_out/pm_$tag.log"
  cut -d, -f1-4 "gpurun_out/pm_$tag/run_kernel_stats.csv" | head -8
done
