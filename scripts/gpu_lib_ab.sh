#!/bin/bash
# One library variant against the default: the codebook-source probe (parity
# against gather + two-source, timing) and a bench A/B, interleaved.
#   gpu_lib_ab.sh <variant name>   (vq-gnn_amd/lib/ab_<name>.so)
set -e
v=$1
out=gpurun_out/${v}_probe.txt
: > $out
for rep in 1 2; do
  for lib in vq-gnn_amd/lib/libvqgnn.so vq-gnn_amd/lib/ab_$v.so; do
    echo "== $lib rep $rep" >> $out
    VQGNN_LIB=$lib timeout -k 10 120 python -u scripts/spmm_cb_probe.py 30 arxiv_gcn >> $out 2>&1
  done
done
grep -E "==|arxiv|identical" $out
TAG=${v}_ab bash scripts/ab_bench.sh "base|| $v|VQGNN_LIB=vq-gnn_amd/lib/ab_$v.so|" "arxiv_gcn:update"
