#!/bin/bash
# Kernel-trace stats of the filtered assign (arxiv_gcn update / feature_update)
# and the fixed-cost probe (VQGNN_ASSIGN_MSWEEP=0: no codeword swept).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-fprof}
mkdir -p $O
for sem in update feature_update; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$sem -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 --config arxiv_gcn --semantics $sem \
    > $O/$sem.json 2> $O/$sem.err || exit 1
  f=$(find $O/$sem -name '*kernel_stats.csv' | head -1)
  echo "== $sem"; grep -i "vq_filter\|near_tie\|vq_assign" $f | cut -d, -f1-5
done
VQGNN_ASSIGN_MSWEEP=0 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/msweep0 -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --steps 20 --warmup 3 --config arxiv_gcn --semantics update \
  > $O/msweep0.json 2> $O/msweep0.err || exit 1
f=$(find $O/msweep0 -name '*kernel_stats.csv' | head -1)
echo "== msweep0"; grep -i "vq_filter\|near_tie" $f | cut -d, -f1-5
