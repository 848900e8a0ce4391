#!/bin/bash
# Two SQ counter passes over the assign kernels of library variants
# ("default" = the in-tree library; "exact" = VQGNN_ASSIGN_EXACT=1; "sweep0"
# = VQGNN_ASSIGN_MSWEEP=0; other names = vq-gnn_amd/lib/ab_<name>.so).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmcc}
mkdir -p $O
P1="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
P2="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_LDS_IDX_ACTIVE"
for n in $1; do
  unset VQGNN_LIB VQGNN_ASSIGN_EXACT VQGNN_ASSIGN_MSWEEP
  case $n in
    default) ;;
    exact) export VQGNN_ASSIGN_EXACT=1 ;;
    sweep0) export VQGNN_ASSIGN_MSWEEP=0 ;;
    *) export VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$n.so ;;
  esac
  i=0
  for CNT in "$P1" "$P2"; do
    i=$((i+1))
    mkdir -p $O/$n
    timeout -s KILL 120 rocprofv3 --pmc $CNT --kernel-trace -d $O/$n/p$i -o run --output-format csv \
      -- python scripts/pmc_target.py vq > $O/$n/p$i.log 2>&1 || { echo "$n rc=$?"; tail -3 $O/$n/p$i.log; exit 1; }
  done
  python scripts/pmc_summary.py $O/$n | grep -A20 "^vq_assign_kernel\|^vq_filter_kernel\|^void vqgnn::vq_filter\|^void vqgnn::vq_assign" | sed "s/^/$n /"
done
