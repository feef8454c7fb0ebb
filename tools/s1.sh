set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 120 ./tools/ablate_mfma 1250000 10 > gpurun_out/abl125.txt 2>&1 && cat gpurun_out/abl125.txt &&
bash tools/gpu_session.sh tests bench c3 --steps 50 -- bench s8 --rows 1250000 --steps 200 --no-cpu-baseline -- prof s8v9 --rows 1250000 --steps 100 --no-cpu-baseline --no-secondary
