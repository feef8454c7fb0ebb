#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"
bash tools/r06_c2t.sh && bash tools/r06_pmc_bf16.sh
