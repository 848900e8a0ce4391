#!/bin/bash
# Codebook-source walker check on one box: its parity tests, the A/B timing
# (default library, and VARIANTS="name ..." libraries ab_<name>.so), then
# (FULL=1) smoke + every -m gpu test via gpu_validate.sh.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05w}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_spmm_task.py -x -v -p no:cacheprovider \
  --timeout 120 --timeout-method thread > $O/spmm_task_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/spmm_task_tests.log | tail -1; [ $rc -ne 0 ] && { tail -30 $O/spmm_task_tests.log; exit $rc; }
timeout -k 10 200 python -u scripts/spmm_walk_ab.py 30 arxiv_gcn > $O/walk_ab.log 2>&1
rc=$?; cat $O/walk_ab.log; [ $rc -ne 0 ] && exit $rc
for v in $VARIANTS; do
  echo "== variant $v"
  VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$v.so timeout -k 10 200 python -u scripts/spmm_walk_ab.py 30 arxiv_gcn > $O/walk_ab_$v.log 2>&1
  rc=$?; grep -E "pipelined|identical" $O/walk_ab_$v.log; [ $rc -ne 0 ] && exit $rc
done
[ "${FULL:-0}" = 1 ] && { TAG=$TAG PART=tests bash scripts/gpu_validate.sh; exit $?; }
exit 0
