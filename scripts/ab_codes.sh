#!/bin/bash
# reddit SpMM: row gathers vs code tiles (library variants x U), one box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
C=${C:-reddit_gcn}
run() {  # name lib U src
  if [ "$2" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/$2; fi
  VQGNN_TASK_U=$3 timeout -k 10 200 python bench.py --config $C --spmm-source $4 --steps 10 --warmup 3 \
    --no-cpu-baseline > gpurun_out/abc_$1.json 2>/dev/null || exit 1
  python -c "import json; d=json.loads(open('gpurun_out/abc_$1.json').read().strip().splitlines()[-1]); print('$1', round(d['ms_per_step'],3), round(d['kernels']['spmm_ms'],3))"
}
for v in $VARIANTS; do IFS=: read n l u s <<< "$v"; run $n $l $u $s; done
