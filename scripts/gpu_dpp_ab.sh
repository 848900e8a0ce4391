#!/bin/bash
# DPP row broadcasts of the task walk's records (default lib) against the
# ds_swizzle build (ab_old): SpMM parity tests, the probe, then bench A/B
set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_spmm_task.py tests/test_gpu_spmm.py > gpurun_out/dpp_tests.txt 2>&1
tail -3 gpurun_out/dpp_tests.txt
out=gpurun_out/dpp_probe.txt
: > $out
for rep in 1 2; do
  for lib in vq-gnn_amd/lib/libvqgnn.so vq-gnn_amd/lib/ab_old.so; do
    echo "== $lib rep $rep" >> $out
    VQGNN_LIB=$lib timeout -k 10 120 python -u scripts/spmm_cb_probe.py 30 arxiv_gcn >> $out 2>&1
  done
done
grep -E "==|arxiv" $out
TAG=dpp_ab bash scripts/ab_bench.sh "dpp|| old|VQGNN_LIB=vq-gnn_amd/lib/ab_old.so|" "arxiv_gcn:update"
