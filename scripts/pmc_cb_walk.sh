#!/bin/bash
# PMC of the codebook-source walk, shipped form (DBG=0) against the
# memory-free probe (DBG=7: no per-edge global loads, no row stores), on the
# probe library ab_cbprobe (scripts/cb_walk_floor.sh); one counter group per run
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/pmc_cbwalk
mkdir -p $O
i=0
for d in 0 7; do
  while read -r line; do
    [ -z "$line" ] && continue
    i=$((i+1))
    VQGNN_LIB=vq-gnn_amd/lib/ab_cbprobe.so VQGNN_TASK_DBG=$d REPS=5 timeout -s KILL 90 \
      rocprofv3 --pmc $line --kernel-trace -d $O/d${d}/p$i -o run --output-format csv \
      -- python scripts/pmc_target.py spmm > $O/d${d}_p$i.log 2>&1
    rc=$?; echo "DBG=$d pass $i ($line) rc=$rc"
    if [ $rc -ne 0 ]; then tail -5 $O/d${d}_p$i.log; exit $rc; fi
  done <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM_WR
LIST
  python scripts/pmc_summary.py $O/d${d} > $O/summary_d${d}.txt
done
