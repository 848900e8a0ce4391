#!/bin/bash
# A/B of the pipelined GAT walker's shape: default (G = 32 lanes per task,
# U = 16 edges per block) vs U = 8 vs G = 16, arxiv_gat, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_gat_shape}; mkdir -p $O
for rep in 1 2; do
  for s in "-" "VQGNN_TASK_U=8" "VQGNN_TASK_G=16"; do
    envs=""; [ "$s" != "-" ] && envs=$s
    env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --config arxiv_gat --steps 30 --warmup 5 \
      > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print('$rep [$s]', 'ms/step %.4f' % d['ms_per_step'], 'gat aggregation ms %.4f' % d['kernels']['spmm_ms'])" | tee -a $O/ab.txt
  done
done
