#!/bin/bash
# Round-3 pass g: the validation pass (smoke, pytest -m gpu, bench, the
# --gpus 2 rehearsal), then an interleaved A/B of the GAT walker
# (ab_gatold.so = the previous spmm_tasks.hip) on arxiv_gat and arxiv_gcn.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${TAG:-r03g} bash scripts/gpu_check.sh || exit $?
bash scripts/ab_libs.sh "old=vq-gnn_amd/lib/ab_gatold.so new=default" --config arxiv_gat --steps 20 --warmup 3 \
  > gpurun_out/${TAG:-r03g}/ab_gat.txt 2>&1; rc=$?; cat gpurun_out/${TAG:-r03g}/ab_gat.txt; exit $rc
