#!/bin/bash
# Round 6: the shipped task SpMM with round-robin dealing for grids of 2^16
# workgroups and more: SpMM parity (incl. reddit), then its time on reddit
# layers 2 and 1 and on arxiv (scripts/spmm_time.py, shipped library).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm_task.py tests/test_gpu_reddit.py -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
for cfg in reddit_gcn reddit_gcn_l1 arxiv_gcn; do
  timeout -k 10 300 python scripts/spmm_time.py $cfg 5 || exit 1
done
