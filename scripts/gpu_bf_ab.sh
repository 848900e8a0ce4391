#!/bin/bash
# Branch-free codebook-source loads (ab_bf: every edge issues the X gather --
# out of range, no access, for codebook edges -- and the LDS read, then a
# select) against the default library: parity of the probe, probe timing,
# bench A/B
set -e
out=gpurun_out/bf_probe.txt
: > $out
for rep in 1 2; do
  for lib in vq-gnn_amd/lib/libvqgnn.so vq-gnn_amd/lib/ab_bf.so; do
    echo "== $lib rep $rep" >> $out
    VQGNN_LIB=$lib timeout -k 10 120 python -u scripts/spmm_cb_probe.py 30 arxiv_gcn >> $out 2>&1
  done
done
grep -E "==|arxiv|identical" $out
TAG=bf_ab bash scripts/ab_bench.sh "base|| bf|VQGNN_LIB=vq-gnn_amd/lib/ab_bf.so|" "arxiv_gcn:update"
