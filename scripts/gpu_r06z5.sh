#!/bin/bash
# Round 6 re-entry: the codebook walk with its first unit's plan words
# requested before the LDS image is staged (ab_hoist) against the walk of
# lib d5afd9ea (ab_old): parity on the task-SpMM suite, scripts/cb_time.py
# interleaved (three rounds, same checksums), then the bench step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z5
mkdir -p $O
L=$PWD/vq-gnn_amd/lib
VQGNN_LIB=$L/ab_hoist.so timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_task.py tests/test_gpu_defer.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_hoist.log 2>&1 || { tail -20 $O/test_hoist.log; exit 1; }
echo "hoist: $(grep -E 'passed|failed' $O/test_hoist.log | tail -1)"
for rep in 1 2 3; do
  for lib in ab_old ab_hoist; do
    VQGNN_LIB=$L/$lib.so timeout -k 10 120 python scripts/cb_time.py arxiv_gcn 30 || exit 1
  done
done
REPS="1 2 3" TAG=r06z5 bash scripts/ab_assign.sh "old hoist" "arxiv_gcn:update" || exit 1
