#!/bin/bash
# Interleaved A/B of library builds on the SpMM alone:
#   ab_spmm.sh "name=path ..." config [config ...]   (path "default" = libvqgnn.so)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
VARS="$1"; shift
for cfg in "$@"; do
  for rep in 1 2; do
    for v in $VARS; do
      p=${v#*=}
      if [ "$p" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/$p; fi
      timeout -k 10 300 python scripts/spmm_time.py $cfg || exit 1
    done
  done
done
