#!/bin/bash
# After a library rebuild: the SpMM / GAT / config GPU tests, then the PMC
# passes (-> pmc_latest.json stamped with the new library), the bench line
# with them and its rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04}
O=gpurun_out/$TAG
mkdir -p $O
log() { echo "== $(date +%T) $1" | tee -a $O/progress.log; }
TESTS=${TESTS:-tests/test_gpu_gat.py tests/test_gpu_spmm_task.py tests/test_gpu_spmm.py tests/test_gpu_configs.py}
log smoke && timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
&& log tests && timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v -p no:cacheprovider --timeout 120 \
     --timeout-method thread > $O/pytest.log 2>&1 \
&& log pmc && TAG=${TAG}_pmc TARGET=step bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 \
&& python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_pmc > $O/pmc_summary.txt \
&& python scripts/pmc_to_json.py gpurun_out/pmc_${TAG}_pmc/summary.json $O/pmc_latest.json arxiv_gcn update > /dev/null \
&& log bench && timeout -k 10 400 python bench.py --steps 30 --warmup 5 --pmc-json $O/pmc_latest.json > $O/bench.log 2>&1 \
&& log rocprof && timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run --output-format csv \
     -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --pmc-json $O/pmc_latest.json > $O/prof_bench.log 2>&1
rc=$?
log "chain rc=$rc"
tail -2 $O/smoke.log
grep -E "passed|failed" $O/pytest.log | tail -1
grep -h '^{' $O/bench.log | cut -c1-300
exit $rc
