#!/bin/bash
# Round 6: (1) parity + timing of the library with the priority changes
# (assign fold, codebook-walk load issue); (2) the two-source task walk with
# the same raised priority while a block's gathers are issued (ab_taskprio)
# against it: scripts/spmm_time.py on arxiv (gathered rows), ppi, reddit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06u
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_taskprio.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm_task.py \
  tests/test_gpu_gat.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_taskprio.log 2>&1 \
  || { tail -20 $O/test_taskprio.log; exit 1; }
echo "taskprio: $(grep -E 'passed|failed' $O/test_taskprio.log | tail -1)"
for r in 1 2; do
  for cfg in arxiv_gcn ppi_sage reddit_gcn; do
    n=30; [ $cfg = reddit_gcn ] && n=5
    timeout -k 10 300 python scripts/spmm_time.py $cfg $n || exit 1
    # (experiments builds map tasks XCD-contiguously by default; the shipped
    # library deals reddit's grid round-robin: the variant is told the same)
    x=1; [ $cfg = reddit_gcn ] && x=0
    VQGNN_TASK_XCD=$x VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_taskprio.so timeout -k 10 300 python scripts/spmm_time.py $cfg $n || exit 1
  done
done
