#!/bin/bash
# Round-3 measurement pass: PMC passes of one arxiv layer step (-> a
# pmc_latest.json stamped with this library and GIT_HEAD), the bench line
# with it (+ CPU baseline), rocprofv3 kernel stats of the same bench, then the
# variant configs.  Every GPU step has its own time limit; the chain stops at
# the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03i}
O=gpurun_out/$TAG
mkdir -p $O
log() { echo "== $(date +%T) $1" | tee -a $O/progress.log; }
log pmc && TAG=${TAG}_pmc TARGET=step bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 \
&& python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_pmc > $O/pmc_summary.txt \
&& python scripts/pmc_to_json.py gpurun_out/pmc_${TAG}_pmc/summary.json $O/pmc_latest.json arxiv_gcn update > /dev/null \
&& log bench && timeout -k 10 400 python bench.py --steps 30 --warmup 5 --pmc-json $O/pmc_latest.json > $O/bench.log 2>&1 \
&& log rocprof && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run --output-format csv \
     -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --pmc-json $O/pmc_latest.json > $O/prof_bench.log 2>&1 \
&& log feature_update && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --semantics feature_update > $O/v_feature_update.log 2>&1 \
&& log gat && timeout -k 10 400 python bench.py --steps 20 --warmup 3 --config arxiv_gat > $O/v_arxiv_gat.log 2>&1 \
&& log ppi && timeout -k 10 400 python bench.py --steps 10 --warmup 2 --config ppi_sage > $O/v_ppi_sage.log 2>&1 \
&& log reddit && timeout -k 10 500 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config reddit_gcn > $O/v_reddit_gcn.log 2>&1 \
&& log reddit_l1 && timeout -k 10 500 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --config reddit_gcn_l1 > $O/v_reddit_gcn_l1.log 2>&1
rc=$?
log "chain rc=$rc"
grep -h '^{' $O/bench.log | cut -c1-300
exit $rc
