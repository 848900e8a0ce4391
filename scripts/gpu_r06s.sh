#!/bin/bash
# Round 6: wave priority in the assign's sweep (s_setprio): raised while a
# wave issues its 8 MFMAs (ab_prio1 / ab_prio3) or while it folds them
# (ab_priofold), against the shipped library; VQ parity on each first.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06s
mkdir -p $O
for v in prio1 prio3 priofold; do
  VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -20 $O/test_$v.log; exit 1; }
  echo "$v: $(grep -E 'passed|failed' $O/test_$v.log | tail -1)"
done
TAG=r06s bash scripts/ab_assign.sh "default prio1 prio3 priofold" "arxiv_gcn:update arxiv_gat:update" || exit 1
