#!/bin/bash
# Interleaved A/B of library builds (VQGNN_LIB) on one box: bench lines per
# variant, repeated; usage: ab_libs.sh "name=path ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="$1"; shift
for rep in 1 2; do
  for v in $VARS; do
    n=${v%%=*}; p=${v#*=}
    if [ "$p" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/$p; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/ab_$n.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.loads(open('gpurun_out/ab_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['roofline']['achieved'],2), round(d['kernels']['vq_update_ms'],4), 'spmm', round(d['kernels']['spmm_ms'],4))"
  done
done
