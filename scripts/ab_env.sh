#!/bin/bash
# Interleaved A/B of environment settings on one box: ab_env.sh "name=VAR=val,VAR2=val ..." [bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="$1"; shift
for rep in 1 2; do
  for v in $VARS; do
    n=${v%%=*}; e=${v#*=}
    envs=(); [ "$e" != "none" ] && IFS=, read -ra envs <<< "$e"
    env "${envs[@]}" timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/abe_$n.json 2>/dev/null || exit 1
    python -c "import json; d=json.loads(open('gpurun_out/abe_$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],4), round(d['kernels']['spmm_ms'],4))"
  done
done
