set -u
for from in 1025 1; do
  VS_LARGE_K_FROM=$from timeout -k 10 200 python -u tools/large_k_bench.py --ks 10,64,100,128,129,200,256,512,1024 --reps 15 > gpurun_out/lk_from_$from.jsonl 2>/dev/null || exit 1
done
for ctx in 1 2; do
  VS_CONTEXTS=$ctx timeout -k 10 300 python -u tools/loadgen_c5.py --transport both --clients 64,256 --seconds 4 --unbatched-clients 0 > gpurun_out/c5_ctx$ctx.jsonl 2>/dev/null || exit 1
done
VS_CONTEXTS=1 timeout -k 10 120 python -u tools/c1_http.py --backend gpu > gpurun_out/c1_ctx1.jsonl 2>/dev/null || exit 1
echo done
