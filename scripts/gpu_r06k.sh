#!/bin/bash
# Round 6: kernel timeline of bench.py's default (overlapped) step and of the
# serial step (rocprofv3 --kernel-trace; scripts/step_timeline.py).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
for ov in auto off; do
  timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace_$ov -o run --output-format csv -- \
    python bench.py --steps 12 --warmup 3 --no-cpu-baseline --overlap $ov > $O/trace_$ov.log 2>&1 \
    || { tail -5 $O/trace_$ov.log; exit 1; }
  f=$(find $O/trace_$ov -name "run_kernel_trace.csv" | head -1)
  cp $f $O/kernel_trace_$ov.csv && rm -rf $O/trace_$ov
  echo "== overlap $ov"
  python scripts/step_timeline.py $O/kernel_trace_$ov.csv bn_cascade_partial 6 2 | tee $O/timeline_$ov.txt | tail -22
done
