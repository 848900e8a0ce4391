#!/bin/bash
# Lanes per task of the two-source task SpMM (VQGNN_TASK_G: 32 -> one float4
# per lane, 16 -> two, 8 -> four; one 128-column tile at F = 128), arxiv
# batch, interleaved (gather + task SpMM timed by scripts/spmm_cb_probe.py)
set -e
out=gpurun_out/task_g_ab.txt
: > $out
for rep in 1 2; do
  for g in 32 16 8; do
    for u in 16 8; do
      echo "== G=$g U=$u rep $rep" >> $out
      VQGNN_TASK_G=$g VQGNN_TASK_U=$u timeout -k 10 120 python -u scripts/spmm_cb_probe.py 30 arxiv_gcn >> $out 2>&1
    done
  done
done
