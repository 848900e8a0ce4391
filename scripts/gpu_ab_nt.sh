#!/bin/bash
# A/B of the SpMM gather cache policy (L2 pollution by one-use rows):
# default vs every gather non-temporal (nt1) vs non-temporal only for
# columns >= 4096 rows from the edge's row (nt2), and the row-end flags packed into
# the broadcast offset (pk: two broadcasts per edge); reddit F = 128 and arxiv.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_nt}; mkdir -p $O
bash scripts/ab_libs.sh "def=default nt1=vq-gnn_amd/lib/ab_nt1.so nt2=vq-gnn_amd/lib/ab_nt2.so pk=vq-gnn_amd/lib/ab_pk.so" \
  --config reddit_gcn --steps 5 --warmup 2 > $O/reddit.txt 2>&1 || { cat $O/reddit.txt; exit 1; }
cat $O/reddit.txt
bash scripts/ab_libs.sh "def=default nt1=vq-gnn_amd/lib/ab_nt1.so nt2=vq-gnn_amd/lib/ab_nt2.so pk=vq-gnn_amd/lib/ab_pk.so" \
  --steps 20 --warmup 5 > $O/arxiv.txt 2>&1; rc=$?; cat $O/arxiv.txt; exit $rc
