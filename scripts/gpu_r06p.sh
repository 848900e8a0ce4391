#!/bin/bash
# Round 6: the 3-layer model step (scripts/bench_model.py) on the final
# library: arxiv GCN (M = 256) and GAT (M = 1024), v2 and hook semantics.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06p
mkdir -p $O
for cfg in arxiv_gcn arxiv_gat; do
  timeout -k 10 300 python -u scripts/bench_model.py --config $cfg --forms v2,hook --steps 20 --warmup 3 \
    > $O/model_$cfg.jsonl 2> $O/model_$cfg.err || { tail -20 $O/model_$cfg.err; exit 1; }
  cat $O/model_$cfg.jsonl
done
