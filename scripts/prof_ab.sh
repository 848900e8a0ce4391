cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for snap in 0 1; do
  VQGNN_TASK_SNAP=$snap timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pab$snap -o run --output-format csv -- python $R/scripts/spmm_once.py arxiv_gcn 20 > $R/gpurun_out/pab$snap.log 2>&1 || exit 1
done
