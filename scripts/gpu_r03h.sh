#!/bin/bash
# Round-3 pass h: GPU tests of the assign's pair-index-in-score sweep, then an
# interleaved A/B against the previous vq_kernels.hip (ab_vqold.so) on
# arxiv_gcn (update), feature_update and arxiv_gat.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-r03h}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_gpu.log | tail -8
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
for a in "" "--semantics feature_update" "--config arxiv_gat"; do
  echo "== $a"
  bash scripts/ab_libs.sh "old=vq-gnn_amd/lib/ab_vqold.so new=default" --steps 30 --warmup 5 $a || exit 1
done 2>&1 | tee $O/ab_assign.txt
