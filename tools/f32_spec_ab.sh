set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
for sp in 1 0; do
  for c in c3f32 c2b256; do
    VS_Q8_SPEC=$sp timeout -k 10 300 python bench.py --config $c --steps 30 --warmup 10 --no-cpu-baseline --no-secondary >> gpurun_out/f32ab_$sp.jsonl 2>> gpurun_out/f32ab.err || exit 1
  done
done
