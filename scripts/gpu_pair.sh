#!/bin/bash
# Pair-SpMM experiments: debug variants (1 no gathers, 2 no stores, 8 no adds)
# and workgroups per CU.  Each step has its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
for v in ${PAIR_VARIANTS:-"X=0" "VQGNN_SPMM_DEBUG=1" "VQGNN_SPMM_DEBUG=8"}; do
  echo "== $v"
  env $v timeout -k 10 120 python scripts/microbench.py pair 2>&1 | grep -E "^pair|wave hot|wave two" || exit 1
done
