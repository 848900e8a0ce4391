#!/bin/bash
# PMC of the split-pass walk probes (scripts/probes/walk3.hip, variants given
# as $1, e.g. "8,108") beside the shipped codebook-source walk, on the arxiv
# bench batch; one counter group per run (rocprofv3 does not split passes).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${1:-8}
O=gpurun_out/pmc_walk3
mkdir -p $O
i=0
while read -r line; do
  [ -z "$line" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $line --kernel-trace -d $O/p$i -o run --output-format csv \
    -- python scripts/walk3_probe.py 2 $V 8 64 > $O/p$i.log 2>&1
  rc=$?; echo "pass $i ($line) rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 $O/p$i.log; exit $rc; fi
done <<'LIST'
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU
SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INSTS_VMEM_WR
TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT
LIST
python scripts/pmc_summary.py $O > $O/summary.txt
