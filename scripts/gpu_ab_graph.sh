#!/bin/bash
# A/B: eager step vs the step captured in a HIP graph (--graph), arxiv_gcn
# and arxiv_gat, interleaved on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab_graph}; mkdir -p $O
for cfg in arxiv_gcn arxiv_gat; do
for rep in 1 2 3; do
  for g in "" "--graph"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --config $cfg --steps 30 --warmup 5 $g \
      > $O/b.json 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
    python -c "import json; d=json.loads([l for l in open('$O/b.json') if l.startswith('{')][-1]); print('$cfg graph=$g', 'ms/step %.4f' % d['ms_per_step'], 'host %.4f' % d.get('host_issue_ms_per_step', 0))" | tee -a $O/ab.txt
  done
done; done
