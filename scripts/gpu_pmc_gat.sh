#!/bin/bash
# PMC passes of the fused GAT aggregation at the arxiv_gat shape (alpha,
# scale, the pipelined task walker, fix-up), one counter group per run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03o_gat} CONFIG=arxiv_gat TARGET=gat PMC_LIST="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD
SQ_INSTS_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS
TCC_HIT TCC_MISS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE" bash scripts/gpu_pmc.sh || exit $?
python scripts/pmc_summary.py gpurun_out/pmc_${TAG:-r03o_gat} > gpurun_out/pmc_${TAG:-r03o_gat}/summary.txt
cat gpurun_out/pmc_${TAG:-r03o_gat}/summary.txt | head -80
