#!/bin/bash
# Assign-kernel iteration pass: smoke -> VQ parity tests -> bench (+ the
# zero-codeword probe) -> the other assign-bound configs.  Each GPU step has
# its own time limit; the chain stops at the first failure.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-assign}
mkdir -p $O
run() { local t=$1; shift; echo "== $(date +%T) $*"; timeout -k 10 $t "$@"; }
run 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log \
&& run 500 python -u -m pytest -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
     ${TESTS:-tests/test_gpu_vq.py tests/test_gpu_layer.py tests/test_gpu_defer.py tests/test_gpu_reddit.py} > $O/pytest.log 2>&1 \
&& tail -2 $O/pytest.log \
&& run 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench.log 2>&1 \
&& VQGNN_ASSIGN_MSWEEP=0 run 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline > $O/bench_msweep0.log 2>&1 \
&& run 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --semantics feature_update > $O/bench_fu.log 2>&1 \
&& run 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline --config arxiv_gat > $O/bench_gat.log 2>&1 \
&& run 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --config ppi_sage > $O/bench_ppi.log 2>&1
rc=$?
echo "chain rc=$rc"
for f in bench bench_msweep0 bench_fu bench_gat bench_ppi; do
  [ -f $O/$f.log ] && grep -h '^{' $O/$f.log | python3 -c "import json,sys
for l in sys.stdin:
    d=json.loads(l); k=d['kernels']
    print('$f', 'ms/step %.4f'%d['ms_per_step'], 'assign us %.1f'%(k['vq_assign']['ms_per_launch']*1e3), 'frac %.3f'%k['vq_assign']['frac'], 'spmm us %.1f'%(k['spmm_ms']*1e3))"
done
exit $rc
