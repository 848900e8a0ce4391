#!/bin/bash
# Round 6: the two-source task SpMM with its workgroups dealt to the XCDs in
# chunks of C (VQGNN_TASK_XCD=C, ab_xcd.so) against contiguous eighths (1, the
# default) and round-robin (0): reddit layer 2, arxiv (gathered rows), ppi.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
X=$PWD/vq-gnn_amd/lib/ab_xcd.so
for r in 1 2; do
  for m in 1 0 16 64 256; do
    VQGNN_LIB=$X VQGNN_TASK_XCD=$m timeout -k 10 300 python scripts/spmm_time.py reddit_gcn 5 | sed "s/^/xcd=$m /" || exit 1
    VQGNN_LIB=$X VQGNN_TASK_XCD=$m timeout -k 10 300 python scripts/spmm_time.py arxiv_gcn 30 | sed "s/^/xcd=$m /" || exit 1
  done
  for m in 1 16 64; do
    VQGNN_LIB=$X VQGNN_TASK_XCD=$m timeout -k 10 300 python scripts/spmm_time.py ppi_sage 30 | sed "s/^/xcd=$m /" || exit 1
  done
done
