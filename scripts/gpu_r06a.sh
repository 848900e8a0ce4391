#!/bin/bash
# Round 6: SpMM unit-start plan reads batched + prefetched, zero image row,
# bad-node weights; parity tests then an interleaved A/B against ab_base.so.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_task.py tests/test_gpu_defer.py tests/test_gpu_gat.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
for rep in 1 2 3; do
  for lib in default vq-gnn_amd/lib/ab_base.so; do
    if [ "$lib" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/$lib; fi
    timeout -k 10 120 python scripts/cb_time.py arxiv_gcn 30 || exit 1
  done
done
