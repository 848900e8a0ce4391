#!/bin/bash
# PMC passes (one counter group per run, kernel-trace only besides --pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc_${TAG:-x}
mkdir -p $OUT
TARGET=${TARGET:-step}
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $line --kernel-trace -T -d $OUT/p$i -o run --output-format csv \
    -- python scripts/pmc_target.py $TARGET > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $OUT/p$i.log; exit $rc; fi
done <<< "${PMC_LIST:-$(cat <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU
SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_IDX_ACTIVE
TCC_HIT TCC_MISS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ
LIST
)}"
