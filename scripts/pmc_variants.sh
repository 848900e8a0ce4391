#!/bin/bash
# One SQ counter pass per library variant (VQGNN_LIB) over the assign kernel
# (scripts/pmc_target.py vq): instruction mix and pipe busy/stall cycles.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmcv}
mkdir -p $O
CNT=${CNT:-"SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU"}
for n in $1; do
  if [ "$n" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$n.so; fi
  mkdir -p $O/$n
  timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace -d $O/$n/p1 -o run --output-format csv \
    -- python scripts/pmc_target.py ${WHAT:-vq} > $O/$n/p1.log 2>&1 || { echo "$n rc=$?"; tail -3 $O/$n/p1.log; exit 1; }
  python scripts/pmc_summary.py $O/$n | grep -A12 "^vq_assign_kernel" | sed "s/^/$n /"
done
