#!/bin/bash
# Counter diagnosis of the reddit SpMM: for the task
# kernel at F = 128 and F = 604 (the tiled path, since removed, was measured
# the same way: profiles/r03_reddit_spmm_pmc.txt), one rocprofv3 pass per
# counter group (kernel-trace only besides --pmc).  Each pass has its own
# time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-pmc_reddit}
mkdir -p $O
LIST="FETCH_SIZE
WRITE_SIZE
TCC_HIT TCC_MISS TCC_EA0_RDREQ TCC_EA0_RDREQ_DRAM
TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT
SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_WAVES"
for cfg in ${CONFIGS:-reddit_gcn reddit_gcn_l1}; do
  for what in ${WHATS:-spmm}; do
    i=0
    while read -r line; do
      [ -z "$line" ] && continue
      i=$((i+1))
      d=$O/${cfg}_${what}/p$i
      mkdir -p $O/${cfg}_${what}
      echo "== $(date +%T) $cfg $what pass $i: $line"
      CONFIG=$cfg REPS=3 timeout -s KILL 240 rocprofv3 --pmc $line --kernel-trace -d $d -o run \
        --output-format csv -- python scripts/pmc_target.py $what > $d.log 2>&1
      rc=$?
      if [ $rc -ne 0 ]; then echo "rc=$rc"; tail -5 $d.log; exit $rc; fi
    done <<< "$LIST"
    python scripts/pmc_summary.py $O/${cfg}_${what} > $O/${cfg}_${what}.txt || exit 1
    # keep the summaries only (the per-dispatch traces exceed what is copied back)
    cp $O/${cfg}_${what}/summary.json $O/${cfg}_${what}.json && rm -rf $O/${cfg}_${what}
  done
done
