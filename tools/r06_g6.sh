#!/bin/bash
# r06: finish A/B (VARS over tools/_ab), one-query tests, C2 split + bench (TAG)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
bash tools/r06_c2var.sh || exit 1
bash tools/r06_c2t.sh
