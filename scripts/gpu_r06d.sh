#!/bin/bash
# Round 6: the assign's resolve with each run's eight k-planes read before its
# chains (ab_rsv.so, WM 1/2 instances): VQ parity tests on the variant, then
# an interleaved assign A/B against the shipped library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06d
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_rsv.so timeout -k 10 500 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py \
  -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_vq_rsv.log 2>&1 || { tail -30 $O/test_vq_rsv.log; exit 1; }
grep -E "passed|failed" $O/test_vq_rsv.log | tail -1
TAG=r06d bash scripts/ab_assign.sh "default rsv" "arxiv_gcn:update arxiv_gcn:feature_update" || exit 1
