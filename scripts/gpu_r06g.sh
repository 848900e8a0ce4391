#!/bin/bash
# Round 6: the reddit SpMM (layer 2, F = 128, the
# two-source task kernel) with XCD-contiguous task ranges (the default:
# xcd_remap, each XCD walks one contiguous eighth of the rows front to back)
# against the dispatcher's round-robin order (ab_xcd.so, VQGNN_TASK_XCD=0):
# time, then L2-miss bytes and L2 hits / misses per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
X=$PWD/vq-gnn_amd/lib/ab_xcd.so
for r in 1 2; do
  timeout -k 10 300 python scripts/spmm_time.py reddit_gcn 5 || exit 1
  VQGNN_LIB=$X VQGNN_TASK_XCD=1 timeout -k 10 300 python scripts/spmm_time.py reddit_gcn 5 || exit 1
  VQGNN_LIB=$X VQGNN_TASK_XCD=0 timeout -k 10 300 python scripts/spmm_time.py reddit_gcn 5 || exit 1
done
for m in 1 0; do
  i=0
  for line in "FETCH_SIZE" "TCC_HIT TCC_MISS GRBM_GUI_ACTIVE"; do
    i=$((i+1)); d=$O/xcd$m/p$i; mkdir -p $O/xcd$m
    echo "== xcd=$m pass $i: $line"
    VQGNN_LIB=$X VQGNN_TASK_XCD=$m CONFIG=reddit_gcn GATHER_ROWS=1 REPS=3 timeout -s KILL 300 \
      rocprofv3 --pmc $line --kernel-trace -d $d -o run --output-format csv -- python scripts/pmc_target.py spmm > $d.log 2>&1 \
      || { echo "rc=$?"; tail -5 $d.log; exit 1; }
  done
  python scripts/pmc_summary.py $O/xcd$m > $O/xcd$m.txt || exit 1
  cp $O/xcd$m/summary.json $O/xcd$m.json && rm -rf $O/xcd$m
  grep -A6 "spmm_task_kernel" $O/xcd$m.txt | head -8
done
