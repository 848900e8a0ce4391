#!/bin/bash
# Round 6: the codebook-source walk on a side stream beside BN statistics +
# assign, the fix-up (with the update's EMA finalize) after both: parity
# tests, then the step interleaved against the serial default.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06e
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_defer.py tests/test_gpu_spmm_task.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
run() {
  local name=$1; shift
  timeout -k 10 150 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err \
    || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],4), d['config'].get('ema_finalize'))"
}
for r in 1 2 3; do
  run serial_$r
  run overlap_$r --overlap
  run overlap_sep_$r --overlap --separate-finalize
  run serial_fu_$r --semantics feature_update
  run overlap_fu_$r --semantics feature_update --overlap
done
