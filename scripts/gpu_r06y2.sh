#!/bin/bash
# Round 6 re-entry: wave priority of the assign's other phases (compile-time
# VQGNN_ASG_ROW_PRIO / _RES_PRIO / _FOLD_PRIO, vq_kernels.hip): the row phase
# raised to 1 (ab_row1) or 2 (ab_row2, above the fold), the resolve to 1
# (ab_res1), the fold to 2 with the row phase at 1 (ab_f2row1), against the
# shipped library (fold at 1); VQ parity on each first, then three
# interleaved rounds (scripts/ab_assign.sh; assign = its HIP-event duration).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y2
mkdir -p $O
for v in row1 res1 row2 f2row1; do
  VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -20 $O/test_$v.log; exit 1; }
  echo "$v: $(grep -E 'passed|failed' $O/test_$v.log | tail -1)"
done
REPS="1 2 3" TAG=r06y2 bash scripts/ab_assign.sh "default row1 res1 row2 f2row1" "arxiv_gcn:update arxiv_gat:update ppi_sage:update" || exit 1
