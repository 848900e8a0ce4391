#!/bin/bash
# Round 5: chunk-outer passes, narrow codebook tiles.  Parity tests (SpMM,
# VQ goldens incl. M = 4,096 and the repeat-launch guard, configs incl. ppi),
# the assign A/B against ab_base.so (round-4 build), chunk settings at ppi,
# and the reddit layer-2 step with the codebook source (M = 1,024) against
# gathered rows.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_spmm_task.py tests/test_gpu_vq.py tests/test_gpu_configs.py tests/test_gpu_bn_fold.py -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread > $O/test.log 2>&1 || { tail -30 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
TAG=r05e_ab bash scripts/ab_assign.sh "default base" "arxiv_gcn:update arxiv_gcn:feature_update arxiv_gat:update" || exit 1
TAG=r05e_ppi bash scripts/ab_assign.sh "default base VQGNN_ASG_CO=0 VQGNN_FLT_CHUNK=1024+VQGNN_FLT_ELDS=1 VQGNN_FLT_CHUNK=1024" "ppi_sage:update" || exit 1
for v in "" "--gather-rows"; do
  timeout -k 10 400 python -u bench.py --config reddit_gcn --no-cpu-baseline --steps 10 --warmup 3 $v > $O/reddit$v.log 2>&1 || { tail -5 $O/reddit$v.log; exit 1; }
  grep '^{' $O/reddit$v.log | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('reddit', '$v', d['config']['aggregation'], 'ms/step %.3f'%d['ms_per_step'], 'spmm ms %.3f'%d['kernels']['spmm_ms'], 'vq ms %.3f'%d['kernels']['vq_update_ms'])"
done
