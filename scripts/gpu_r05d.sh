#!/bin/bash
# Round-5 batch: the overlapped-hook parity test, the hook-form model step
# A/B (arxiv GCN and GAT), and the assign PMC passes at ppi / arxiv_gat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_layer.py -x -v -p no:cacheprovider -k side_stream \
  --timeout 120 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
for cfg in arxiv_gcn arxiv_gat; do
  timeout -k 10 300 python -u scripts/bench_model.py --config $cfg --forms v2,hook,hook_overlap,hook,hook_overlap \
    > $O/model_$cfg.jsonl 2>&1 || { tail -5 $O/model_$cfg.jsonl; exit 1; }
  grep '^{' $O/model_$cfg.jsonl | python3 -c "import sys,json; [print(d['config'], d['form'], round(d['ms_per_step'],3)) for d in map(json.loads, sys.stdin)]"
done
CONFIG=ppi_sage TAG=r05_ppi bash scripts/pmc_assign_cmp.sh "default sweep0" > $O/ppi_pmc.txt 2>&1 || exit 1
CONFIG=arxiv_gat TAG=r05_gat bash scripts/pmc_assign_cmp.sh "default sweep0" > $O/gat_pmc.txt 2>&1 || exit 1
exit 0
