#!/bin/bash
# Round 6: cache policy of the SpMM walks' streaming accesses -- output-row
# stores with sc1 (the line leaves the XCD's L2) or nt, record loads with nt
# -- against the shipped library (ab_st16, ab_st2, ab_rec2, ab_st16rec2:
# -DVQGNN_OUT_AUX / -DVQGNN_REC_AUX).  Parity of one variant on the task-SpMM
# suite, then the codebook-source aggregation on arxiv (scripts/cb_time.py)
# and the two-source task SpMM on reddit layer 2 (scripts/spmm_time.py),
# interleaved, same checksums.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06w
mkdir -p $O
L=$PWD/vq-gnn_amd/lib
VQGNN_LIB=$L/ab_st16rec2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_task.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_st16rec2.log 2>&1 || { tail -20 $O/test_st16rec2.log; exit 1; }
echo "st16rec2: $(grep -E 'passed|failed' $O/test_st16rec2.log | tail -1)"
for rep in 1 2; do
  for lib in libvqgnn ab_st16 ab_st2 ab_rec2 ab_st16rec2; do
    VQGNN_LIB=$L/$lib.so timeout -k 10 120 python scripts/cb_time.py arxiv_gcn 30 || exit 1
  done
done
for rep in 1 2; do
  for lib in libvqgnn ab_st16 ab_rec2 ab_st16rec2; do
    VQGNN_LIB=$L/$lib.so timeout -k 10 300 python scripts/spmm_time.py reddit_gcn 5 || exit 1
  done
done
