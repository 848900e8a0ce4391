#!/bin/bash
# Overlap probe sweep (SpMM on a side stream beside the VQ update) at several
# assign occupancies, plus the SpMM variants.  Each GPU step has its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ov
set -o pipefail
run() { echo "== $*"; timeout -k 10 120 "$@" 2>&1 | grep -v amdgpu.ids; }
run python scripts/overlap_probe.py > gpurun_out/ov/auto.log \
&& VQGNN_ASG_TARGET=512 run python scripts/overlap_probe.py > gpurun_out/ov/t512.log \
&& VQGNN_ASG_TARGET=256 run python scripts/overlap_probe.py > gpurun_out/ov/t256.log \
&& OV_PRIO=-1 VQGNN_ASG_TARGET=512 run python scripts/overlap_probe.py > gpurun_out/ov/t512p.log \
&& run python scripts/microbench.py codes > gpurun_out/ov/codes.log \
&& VQGNN_SPMM_FLAT=16 run python scripts/microbench.py spmm > gpurun_out/ov/flat16.log \
&& VQGNN_SPMM_FLAT=32 run python scripts/microbench.py spmm > gpurun_out/ov/flat32.log \
&& run python scripts/microbench.py spmm > gpurun_out/ov/wave.log
rc=$?
cat gpurun_out/ov/*.log
exit $rc
