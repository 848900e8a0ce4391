#!/bin/bash
# Round-3 pass j: rocprofv3 kernel stats of the arxiv_gat bench (the GAT
# walker's own time) and the assign decomposition probe on the final build
# (full sweep and VQGNN_ASSIGN_MSWEEP=0).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r03j}; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O/prof_gat -o run --output-format csv \
  -- python bench.py --config arxiv_gat --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_gat.log 2>&1 || exit $?
timeout -k 10 200 python scripts/assign_probe.py > $O/probe.txt 2>&1 || exit $?
VQGNN_ASSIGN_MSWEEP=0 timeout -k 10 200 python scripts/assign_probe.py > $O/probe_msweep0.txt 2>&1 || exit $?
cut -d, -f1-4 $O/prof_gat/run_kernel_stats.csv | cut -c1-120; cat $O/probe.txt $O/probe_msweep0.txt
