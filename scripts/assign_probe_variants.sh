#!/bin/bash
# scripts/assign_probe.py on library variants (VQGNN_LIB), with and without
# the codeword sweep:  assign_probe_variants.sh "default name ..." [W]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for n in $1; do
  if [ "$n" = "default" ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$n.so; fi
  for ms in all 0; do
    if [ "$ms" = all ]; then unset VQGNN_ASSIGN_MSWEEP; else export VQGNN_ASSIGN_MSWEEP=$ms; fi
    echo "== lib $n msweep $ms"
    W=${2:-8} timeout -k 10 180 python -u scripts/assign_probe.py || exit 1
  done
done
