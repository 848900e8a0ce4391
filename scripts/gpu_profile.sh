#!/bin/bash
# Kernel-trace profile of the bench (no PMC counters in this pass).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 rocprofv3 --kernel-trace --stats -T -d gpurun_out/$TAG -o run --output-format csv \
  -- python bench.py --steps ${STEPS:-20} --warmup 5 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/$TAG/bench.log 2>&1
rc=$?; echo "rocprof rc=$rc"; tail -2 gpurun_out/$TAG/bench.log
find gpurun_out/$TAG -name "*stats*" | head
exit $rc
