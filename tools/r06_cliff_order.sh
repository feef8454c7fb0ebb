#!/bin/bash
# r06: the clustered cliff scenario with the engines created in both orders
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(pwd)}"; mkdir -p gpurun_out
for o in 0 1; do
  T_OFF_FIRST=$o timeout -k 10 400 python -u -m pytest -q --timeout 380 --timeout-method thread "tests/test_q8_spec_cliff_gpu.py::test_outlier_queries_do_not_poison_later_batches[clusters]" > gpurun_out/r06_cliff_order_$o.log 2>&1
  echo "order $o rc $?"; cp gpurun_out/spec_cliff_clusters.json gpurun_out/r06_cliff_order_$o.json
done
