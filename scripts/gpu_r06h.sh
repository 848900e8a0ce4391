#!/bin/bash
# Round 6: the overlapped step again, with the walk's output and workspace
# allocated on the compute stream (the first form allocated them on the side
# stream and marked them with record_stream: 0.208-0.223 ms, profiles/
# r06e_overlap_ab.txt), against the serial step and the whole-aggregation-on-
# the-side form (--overlap-whole).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_defer.py -x -q -p no:cacheprovider \
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
  run whole_$r --overlap-whole
  run serial_sep_$r --separate-finalize
done
