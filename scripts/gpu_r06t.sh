#!/bin/bash
# Round 6: (1) the assign with raised wave priority during the sweep's fold
# (ab_priofold) against the shipped library, three interleaved rounds on
# arxiv, arxiv_gat and ppi; (2) the codebook walk with raised priority while
# a block's loads are issued (ab_cbprio), scripts/cb_time.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06t
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_cbprio.so timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_task.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_cbprio.log 2>&1 || { tail -20 $O/test_cbprio.log; exit 1; }
echo "cbprio: $(grep -E 'passed|failed' $O/test_cbprio.log | tail -1)"
for rep in 1 2 3; do
  for lib in default vq-gnn_amd/lib/ab_cbprio.so; do
    if [ "$lib" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/$lib; fi
    timeout -k 10 120 python scripts/cb_time.py arxiv_gcn 30 || exit 1
  done
done
unset VQGNN_LIB
TAG=r06t bash scripts/ab_assign.sh "default priofold" "arxiv_gcn:update arxiv_gat:update ppi_sage:update arxiv_gcn:feature_update" || exit 1
