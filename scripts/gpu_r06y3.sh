#!/bin/bash
# Round 6 re-entry: the assign's phase priorities around the new default
# (fold 2, row phase 1): fold 3 / row 2 (ab_f3row2: the same order of levels, a noise control), fold 2 / row 2
# (ab_f2row2: fold and row phase level), the resolve at 1 too (ab_res1b), the outputs + EMA statistics
# phase raised to 1 (ab_out1); VQ parity on each first, then three
# interleaved rounds (scripts/ab_assign.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y3
mkdir -p $O
for v in f3row2 out1 f2row2 res1b; do
  VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_$v.log 2>&1 || { tail -20 $O/test_$v.log; exit 1; }
  echo "$v: $(grep -E 'passed|failed' $O/test_$v.log | tail -1)"
done
REPS="1 2 3" TAG=r06y3 bash scripts/ab_assign.sh "default f3row2 out1 f2row2 res1b" "arxiv_gcn:update arxiv_gat:update" || exit 1
