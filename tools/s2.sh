set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do for fl in 0 4 3; do
VS_SAMPLE_FLOOR=$fl timeout -k 10 200 python -u bench.py --rows 1250000 --steps 300 --no-cpu-baseline --no-secondary > gpurun_out/ab_$fl.json 2>/dev/null || exit 1
python -c "import json; d=json.load(open('gpurun_out/ab_$fl.json')); print('floor $fl', d['ms_per_step'], d['roofline']['kernel_ms'])"
done; done
