set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for f in 0 1; do
for cfg in "200000 5000" "200000 1000" "20000 1000" "10000000 1000"; do
set -- $cfg
VS_RSEL_FUSED=$f VS_SWEEP_ROWS=$1 VS_SWEEP_DTYPE=bf16 VS_SWEEP_K=$2 timeout -k 10 150 rocprofv3 --kernel-trace --stats -d "$PWD/gpurun_out/rq_${f}_$1_$2" -o run --output-format csv -- python tools/tiny_sweep.py > gpurun_out/rq_${f}_$1_$2.log 2>&1 || exit 1
rm -f gpurun_out/rq_${f}_$1_$2/run_kernel_trace.csv
done
done
