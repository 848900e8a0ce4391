#!/bin/bash
# Round 6 re-entry: the codebook walk's consume phase (fma chain, row stores)
# at wave priority 2, above the block loads' 1 (ab_cons2, -DVQGNN_CB_CONS_PRIO=2),
# against the shipped library: parity on the task-SpMM suite, then
# scripts/cb_time.py interleaved, three rounds, and the bench step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y4
mkdir -p $O
L=$PWD/vq-gnn_amd/lib
VQGNN_LIB=$L/ab_cons2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_task.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_cons2.log 2>&1 || { tail -20 $O/test_cons2.log; exit 1; }
echo "cons2: $(grep -E 'passed|failed' $O/test_cons2.log | tail -1)"
for rep in 1 2 3; do
  for lib in libvqgnn ab_cons2; do
    VQGNN_LIB=$L/$lib.so timeout -k 10 120 python scripts/cb_time.py arxiv_gcn 30 || exit 1
  done
done
REPS="1 2" TAG=r06y4 bash scripts/ab_assign.sh "default cons2" "arxiv_gcn:update" || exit 1
