set -u
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 200 ./tools/ablate_mfma 10000000 4 > gpurun_out/abl10m.txt 2>&1 && grep -E "clocks|main" gpurun_out/abl10m.txt &&
timeout -k 10 200 ./tools/ablate_mfma 1250000 8 > gpurun_out/abl125.txt 2>&1 && grep -E "clocks|main" gpurun_out/abl125.txt
