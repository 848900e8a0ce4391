#!/bin/bash
# Round 6: (1) SpMM unit-start plan reads + zero image row: parity tests and
# an interleaved A/B against ab_base.so; (2) the assign's repeat-launch test at
# 13-32 branches x 30,000 rows, once on the shipped build (SLP-packed resolve
# in the general instance) and once on ab_noslp.so (no packed FP32), then the
# assign A/B of the two.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_task.py tests/test_gpu_defer.py tests/test_gpu_gat.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test_spmm.log 2>&1 || { tail -30 $O/test_spmm.log; exit 1; }
grep -E "passed|failed" $O/test_spmm.log | tail -1
for rep in 1 2 3; do
  for lib in default vq-gnn_amd/lib/ab_base.so; do
    if [ "$lib" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/$lib; fi
    timeout -k 10 120 python scripts/cb_time.py arxiv_gcn 30 || exit 1
  done
done
unset VQGNN_LIB
timeout -k 10 300 python -u -m pytest tests/test_gpu_vq.py -k "repeat_launches" -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test_repeat_slp.log 2>&1
echo "repeat tests, shipped (SLP) build: rc=$?"; grep -E "passed|failed|mismatch" $O/test_repeat_slp.log | tail -8
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_noslp.so timeout -k 10 300 python -u -m pytest tests/test_gpu_vq.py -k "repeat_launches" -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test_repeat_noslp.log 2>&1
echo "repeat tests, no-SLP build: rc=$?"; grep -E "passed|failed|mismatch" $O/test_repeat_noslp.log | tail -8
TAG=r06b bash scripts/ab_assign.sh "default noslp" "arxiv_gcn:update arxiv_gat:update" || exit 1
