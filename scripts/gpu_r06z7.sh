#!/bin/bash
# Round 6 re-entry: the assign with its first row requested before the
# codebook is staged (ab_anew) against lib e4055e60's assign (ab_aold): VQ +
# config parity, then three interleaved rounds (scripts/ab_assign.sh) on
# arxiv and arxiv_gat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z7
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_anew.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_anew.log 2>&1 || { tail -20 $O/test_anew.log; exit 1; }
echo "anew: $(grep -E 'passed|failed' $O/test_anew.log | tail -1)"
REPS="1 2 3" TAG=r06z7 bash scripts/ab_assign.sh "aold anew" "arxiv_gcn:update arxiv_gat:update" || exit 1
