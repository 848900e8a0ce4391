#!/bin/bash
# Task-plan shape A/B on the SpMM alone: K (edges per task) x the snap
# threshold (rows up to SNAP edges are never cut; 1 = K/2).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for cfg in "$@"; do for rep in 1 2; do
  for ks in 64:1 64:64 64:128 64:256 32:64 32:128 128:1 128:256; do
    K=${ks%%:*}; S=${ks#*:}
    VQGNN_TASK_K=$K VQGNN_TASK_SNAP=$S timeout -k 10 120 python scripts/spmm_time.py $cfg | sed "s/^/K=$K snap=$S /" || exit 1
  done
done; done
