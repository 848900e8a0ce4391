#!/bin/bash
# Full validation of the library on one box: smoke, every -m gpu test, then
# (PART=measure) the PMC passes of the bench step (-> pmc_latest.json stamped
# with this library; PMC_JSON=<file>: reuse that stamp), the bench line with
# them, its rocprofv3 kernel stats and the config variants.  Every GPU step has its own time limit; a crash / abort /
# time-limit kill (exit > 1) ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r04v}
O=gpurun_out/$TAG
mkdir -p $O
log() { echo "== $(date +%T) $1" | tee -a $O/progress.log; }
stop() { log "stop rc=$1"; exit $1; }
if [ "${PART:-tests}" = tests ]; then
  log smoke
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
  rc=$?; tail -1 $O/smoke.log; [ $rc -gt 1 ] && stop $rc
  log pytest
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 200 \
    --timeout-method thread > $O/pytest_gpu.log 2>&1
  rc=$?; grep -E "passed|failed" $O/pytest_gpu.log | tail -1; grep -E "FAILED|Error" $O/pytest_gpu.log | head -5
  stop $rc
fi
if [ -n "$PMC_JSON" ]; then          # counters of this library collected already
  cp "$PMC_JSON" $O/pmc_latest.json
else
  log pmc
  TAG=${TAG}_pmc TARGET=step bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 || stop $?
  python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_pmc > $O/pmc_summary.txt
  python scripts/pmc_to_json.py gpurun_out/pmc_${TAG}_pmc/summary.json $O/pmc_latest.json arxiv_gcn update > /dev/null
fi
log bench
timeout -k 10 400 python -u bench.py --steps 30 --warmup 5 --pmc-json $O/pmc_latest.json > $O/bench.log 2>&1 || stop $?
grep -h '^{' $O/bench.log | cut -c1-400
log rocprof
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run --output-format csv \
  -- python bench.py --steps 30 --warmup 5 --no-cpu-baseline --pmc-json $O/pmc_latest.json > $O/prof_bench.log 2>&1 || stop $?
log variants
for v in "--config arxiv_gcn --semantics feature_update" "--config arxiv_gat" "--config ppi_sage" "--config reddit_gcn"; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 $v >> $O/bench_variants.jsonl.log 2>&1 || stop $?
done
grep -h '^{' $O/bench_variants.jsonl.log | cut -c1-300
stop 0
