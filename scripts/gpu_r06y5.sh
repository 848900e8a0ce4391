#!/bin/bash
# Round 6 re-entry: the assign's index / code stores issued one iteration
# later, after the next row's loads were waited for (ab_defer,
# -DVQGNN_ASG_DEFER_STORES=1), against the shipped library: VQ parity, then
# three interleaved rounds (scripts/ab_assign.sh) on arxiv, arxiv_gat, ppi.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y5
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_defer.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_defer.log 2>&1 || { tail -20 $O/test_defer.log; exit 1; }
echo "defer: $(grep -E 'passed|failed' $O/test_defer.log | tail -1)"
REPS="1 2 3" TAG=r06y5 bash scripts/ab_assign.sh "default defer" "arxiv_gcn:update arxiv_gat:update ppi_sage:update" || exit 1
