#!/bin/bash
# Round 6: the fused assign instances with a static single chunk (ab_nch.so:
# fewer SGPR spills, 119 VGPRs): VQ parity on the variant, then the assign A/B.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_nch.so timeout -k 10 500 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py \
  -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_vq_nch.log 2>&1 || { tail -30 $O/test_vq_nch.log; exit 1; }
grep -E "passed|failed" $O/test_vq_nch.log | tail -1
TAG=r06f bash scripts/ab_assign.sh "default nch" "arxiv_gcn:update arxiv_gcn:feature_update" || exit 1
