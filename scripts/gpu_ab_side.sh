#!/bin/bash
# A/B: codeword gather on a side stream beside BN + assign (a bench.py patch,
# reverted after this A/B: profiles/r03g_gather_side_stream_ab.txt) vs in
# order (VQGNN_BENCH_GATHER_SIDE=0), arxiv_gcn and arxiv_gat, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_side}; mkdir -p $O
for cfg in arxiv_gcn arxiv_gat; do
for rep in 1 2 3; do
  for v in 1 0; do
    VQGNN_BENCH_GATHER_SIDE=$v timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg \
      --steps 30 --warmup 5 > $O/b_${cfg}_$v.json 2> $O/b_${cfg}_$v.err || { tail -5 $O/b_${cfg}_$v.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/b_${cfg}_$v.json') if l.startswith('{')][-1]); print('$cfg side=$v', 'ms/step %.4f' % d['ms_per_step'], d['config']['gather_stream'])" | tee -a $O/ab.txt
  done
done; done
