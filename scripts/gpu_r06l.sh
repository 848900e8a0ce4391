#!/bin/bash
# Round 6: the overlapped step with the walk queued after the update's
# BatchNorm launches (deferred walk, the new default) against the walk queued
# first (--walk-first, the previous default) and the serial step, each also
# without the assign's timing events (--no-kernel-events); parity first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
run() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err \
    || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],4))"
}
for r in 1 2 3; do
  run deferred_$r
  run walkfirst_$r --walk-first
  run serial_$r --overlap off
  run deferred_noev_$r --no-kernel-events
  run serial_noev_$r --overlap off --no-kernel-events
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv -- \
  python bench.py --steps 12 --warmup 3 --no-cpu-baseline > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
f=$(find $O/trace -name "run_kernel_trace.csv" | head -1)
cp $f $O/kernel_trace.csv && rm -rf $O/trace
python scripts/step_timeline.py $O/kernel_trace.csv bn_cascade_partial 6 2 | tail -16
