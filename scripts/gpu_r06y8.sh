#!/bin/bash
# Round 6 re-entry: the chunk-outer assign instances (ppi, M = 4,096) with the
# single-pass instances' wave priorities (fold 2, row phase 1; ab_coprio,
# -DVQGNN_ASG_CO_PRIO=1), now that dead waves leave the row loop, against the
# shipped library (fold 1, row phase 0 there): VQ + config parity, then
# three interleaved rounds on ppi (scripts/ab_assign.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06y8
mkdir -p $O
VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_coprio.so timeout -k 10 400 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread > $O/test_coprio.log 2>&1 || { tail -20 $O/test_coprio.log; exit 1; }
echo "coprio: $(grep -E 'passed|failed' $O/test_coprio.log | tail -1)"
REPS="1 2 3" TAG=r06y8 bash scripts/ab_assign.sh "default coprio" "ppi_sage:update" || exit 1
