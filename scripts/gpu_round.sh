#!/bin/bash
# One measurement pass for profiles/: smoke -> pytest -m gpu -> bench ->
# rocprofv3 kernel-trace stats of the bench -> PMC passes of one layer step
# -> profiles/pmc_latest.json.  Every GPU step has its own time limit and the
# chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r01}
O=gpurun_out/$TAG
mkdir -p $O
step() { echo "== $1"; }
step smoke && timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 \
&& step pytest && timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider > $O/pytest_gpu.log 2>&1 \
&& step bench && timeout -k 10 600 python bench.py --steps ${STEPS:-30} --warmup 5 > $O/bench.log 2>&1 \
&& step rocprof && timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d $O/prof -o run --output-format csv \
     -- python bench.py --steps ${STEPS:-30} --warmup 5 --no-cpu-baseline > $O/prof_bench.log 2>&1 \
&& step pmc && TAG=${TAG}_pmc TARGET=step bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1 \
&& python scripts/pmc_summary.py gpurun_out/pmc_${TAG}_pmc > $O/pmc_summary.txt \
&& python scripts/pmc_to_json.py gpurun_out/pmc_${TAG}_pmc/summary.json $O/pmc_latest.json arxiv_gcn update > /dev/null \
&& step variants && timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --semantics feature_update > $O/bench_feature_update.log 2>&1 \
&& timeout -k 10 300 python bench.py --steps 20 --warmup 3 --config arxiv_gat > $O/bench_arxiv_gat.log 2>&1 \
&& timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu-baseline --config ppi_sage > $O/bench_ppi_sage.log 2>&1 \
&& timeout -k 10 300 python scripts/bench_subgraph.py > $O/bench_subgraph.log 2>&1
rc=$?
echo "rc=$rc"
tail -2 $O/smoke.log; tail -2 $O/pytest_gpu.log; grep '^{' $O/bench.log | tail -1
exit $rc
