#!/bin/bash
# Round 6 re-entry: the assign's dead waves leave the row loop (ab_tail,
# -DVQGNN_ASG_TAIL_EXIT=1: a part's last iteration is partial, 172 of 512 rows
# at arxiv, and its dead waves swept clamped rows), against the shipped
# library: VQ + config parity, then three interleaved rounds
# (scripts/ab_assign.sh) on arxiv, arxiv_gat, ppi.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y6
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_tail.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_tail.log 2>&1 || { tail -20 $O/test_tail.log; exit 1; }
echo "tail: $(grep -E 'passed|failed' $O/test_tail.log | tail -1)"
REPS="1 2 3" TAG=r06y6 bash scripts/ab_assign.sh "default tail" "arxiv_gcn:update arxiv_gat:update ppi_sage:update" || exit 1
