set -o pipefail
export VS_SWEEP_ROWS=2000,20000,200000,1000000 VS_SWEEP_K=10,32,50,100,128
for f in 129 33; do
  VS_LARGE_K_FROM=$f timeout -k 10 200 python tools/tiny_sweep.py >> gpurun_out/sweep_lk.jsonl || exit 1
done
