#!/bin/bash
# GPU validation pass: smoke -> pytest -m gpu -> bench -> the N = 2 bench
# rehearsal on one GPU (gloo, both ranks on cuda:0).  Every GPU step has its
# own time limit; a crash / abort / time-limit kill (exit > 1) ends the
# script, plain test failures (exit 1) continue.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-check}
mkdir -p $O
STEPS=${STEPS:-20}
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $O/smoke.log
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread ${PYTEST_ARGS} > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -15
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 400 python -u bench.py --steps $STEPS --warmup 5 ${BENCH_ARGS} > $O/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; grep '^{' $O/bench.log | cut -c1-300
if [ $rc -gt 1 ]; then exit $rc; fi
VQGNN_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -u bench.py --gpus 2 --backend gloo --steps 10 \
  --warmup 3 --no-cpu-baseline > $O/bench_gpus2_gloo.log 2>&1
rc=$?; echo "bench --gpus 2 (gloo, one device) rc=$rc"; grep '^{' $O/bench_gpus2_gloo.log | cut -c1-300
exit $rc
