#!/bin/bash
# GAT normalisation by reciprocal: GAT / config tests, GAT A/B against the
# previous library (ab_gatdiv.so), then the PMC stamp + bench of this library.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03p}; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gat.py tests/test_gpu_configs.py -m gpu -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { grep -E "FAIL|Error" $O/pytest.log | head; exit 1; }
grep -E "passed|failed" $O/pytest.log | tail -1
bash scripts/ab_libs.sh "old=vq-gnn_amd/lib/ab_gatdiv.so new=default" --config arxiv_gat --steps 30 --warmup 5 \
  > $O/ab_gat.txt 2>&1 || exit 1
cat $O/ab_gat.txt
TAG=${TAG:-r03p} bash scripts/gpu_stamp.sh
