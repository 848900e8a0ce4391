#!/bin/bash
# Records three blocks ahead (ab_rec3) against one block ahead (ab_cbprobe),
# both with the walk-floor knobs of scripts/cb_walk_floor.sh
set -e
out=gpurun_out/cb_walk_rec.txt
: > $out
for rep in 1 2; do
  for lib in ab_cbprobe ab_rec3; do
    for d in 0 7; do
      echo "== $lib DBG=$d rep $rep" >> $out
      VQGNN_LIB=vq-gnn_amd/lib/$lib.so VQGNN_TASK_DBG=$d timeout -k 10 120 \
        python -u scripts/spmm_cb_probe.py 30 arxiv_gcn >> $out 2>&1
    done
  done
done
