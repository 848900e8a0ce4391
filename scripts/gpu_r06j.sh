#!/bin/bash
# Round 6: the two-source task SpMM with the dispatcher's round-robin order
# (VQGNN_TASK_XCD=0, ab_xcd.so) against XCD-contiguous task ranges (the
# default) on every config that runs it: reddit layers 2 and 1, ppi, and the
# arxiv batch (gathered rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
X=$PWD/vq-gnn_amd/lib/ab_xcd.so
for cfg in arxiv_gcn ppi_sage reddit_gcn_l1; do
  for r in 1 2; do
    VQGNN_LIB=$X VQGNN_TASK_XCD=1 timeout -k 10 300 python scripts/spmm_time.py $cfg 5 || exit 1
    VQGNN_LIB=$X VQGNN_TASK_XCD=0 timeout -k 10 300 python scripts/spmm_time.py $cfg 5 || exit 1
  done
done
# the overlapped step's kernel timeline (default library, default flags)
O=gpurun_out/r06j
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
python scripts/step_timeline.py $f bn_cascade_partial 3 > $O/timeline.txt && cat $O/timeline.txt
rm -rf $O/trace
