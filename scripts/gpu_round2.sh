#!/bin/bash
# Round-2 measurement pass for profiles/: bench (+ CPU baseline) -> rocprofv3
# kernel stats of the bench -> PMC passes of one layer step -> a TA pass on
# the SpMM -> variant configs (with CPU baselines) -> 3-layer model totals.
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
O=gpurun_out/$TAG
mkdir -p $O
log() { echo "== $(date +%T) $1" | tee -a $O/progress.log; }
log bench && timeout -k 10 400 python bench.py --steps 30 --warmup 5 > $O/bench.log 2>&1 \
&& log rocprof && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run --output-format csv \
     -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1 \
&& log pmc && TAG=${TAG}_pmc TARGET=step bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 \
&& python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_pmc > $O/pmc_summary.txt \
&& python scripts/pmc_to_json.py gpurun_out/pmc_${TAG}_pmc/summary.json $O/pmc_latest.json arxiv_gcn update > /dev/null \
&& log variants && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --semantics feature_update > $O/v_feature_update.log 2>&1 \
&& log gat && timeout -k 10 400 python bench.py --steps 20 --warmup 3 --config arxiv_gat > $O/v_arxiv_gat.log 2>&1 \
&& log ppi && timeout -k 10 400 python bench.py --steps 10 --warmup 2 --config ppi_sage > $O/v_ppi_sage.log 2>&1 \
&& log reddit && timeout -k 10 500 python bench.py --steps 10 --warmup 2 --config reddit_gcn > $O/v_reddit_gcn.log 2>&1 \
&& log reddit_l1 && timeout -k 10 500 python bench.py --steps 5 --warmup 2 --config reddit_gcn_l1 > $O/v_reddit_gcn_l1.log 2>&1 \
&& log model && timeout -k 10 300 python scripts/bench_model.py --steps 20 > $O/model.log 2>&1 \
&& timeout -k 10 300 python scripts/bench_model.py --config arxiv_gat --steps 10 > $O/model_gat.log 2>&1
rc=$?
log "chain rc=$rc"
if [ $rc -eq 0 ]; then
  log ta && timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max --kernel-trace -d $O/pmc_ta -o run --output-format csv \
    -- python scripts/pmc_target.py spmm > $O/pmc_ta.log 2>&1
  log "ta rc=$?"
fi
grep -h '^{' $O/bench.log | cut -c1-200
exit $rc
