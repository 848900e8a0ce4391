#!/bin/bash
# Walk-floor probes of the codebook-source SpMM (library variant ab_cbprobe,
# built by scripts/build_variant.sh from a copy of spmm_tasks.hip with two
# measurement knobs; results invalid except at DBG=0):
#   VQGNN_TASK_DBG=1: no row stores (every knob below: results invalid)
#   VQGNN_TASK_DBG=2: no code loads (codebook edges read image row from the offset bits)
#   VQGNN_TASK_DBG=4: X edges read an LDS image row instead of their global X row
#   VQGNN_TASK_DBG=6: both (every edge from LDS, no per-edge global load)
# Usage: cb_walk_floor.sh "0 2 4 6" [outfile]
set -e
out=${2:-gpurun_out/cb_walk_floor.txt}
: > $out
for rep in 1 2; do
  for d in ${1:-0 2 4 6}; do
    echo "== DBG=$d rep $rep" >> $out
    VQGNN_LIB=vq-gnn_amd/lib/ab_cbprobe.so VQGNN_TASK_DBG=$d timeout -k 10 120 \
      python -u scripts/spmm_cb_probe.py 30 arxiv_gcn >> $out 2>&1
  done
done
