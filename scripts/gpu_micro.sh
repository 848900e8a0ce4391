#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
i=0
while read -r envs; do
  [ -z "$envs" ] && continue
  i=$((i+1))
  env $envs timeout -k 10 300 python scripts/microbench.py ${MB_WHAT:-all} > gpurun_out/micro_$i.log 2>&1
  rc=$?; echo "== [$envs] rc=$rc"; grep -v amdgpu.ids gpurun_out/micro_$i.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done <<< "${VARIANTS:-VQGNN_SPMM_MODE=0}"
