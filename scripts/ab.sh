#!/bin/bash
# A/B of two builds of libvqgnn.so on one box: alternating runs of
# scripts/microbench.py $MB_WHAT with VQGNN_LIB = ab/libvqgnn_prev.so and the
# in-tree build.  Every GPU step has its own time limit; stops at a failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for r in 1 2; do
  for L in ab/libvqgnn_prev.so vq-gnn_amd/lib/libvqgnn.so; do
    VQGNN_LIB=$PWD/$L timeout -k 10 300 python scripts/microbench.py ${MB_WHAT:-vq} > gpurun_out/ab.log 2>&1
    rc=$?; echo "== $L rc=$rc"; grep -v amdgpu.ids gpurun_out/ab.log
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
