#!/bin/bash
# TA occupancy of the codebook-source SpMM walks (TA_BUSY_avr/max per
# dispatch) for the default library and VARIANTS="name ..." (ab_<name>.so),
# then the interleaved A/B timing of each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r05ta}
O=gpurun_out/$TAG
mkdir -p $O
for v in default $VARIANTS; do
  if [ $v = default ]; then unset VQGNN_LIB; else export VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$v.so; fi
  echo "== $v"
  timeout -k 10 200 python -u scripts/spmm_walk_ab.py 30 arxiv_gcn > $O/walk_ab_$v.log 2>&1 || exit $?
  grep -E "walk|walker|gather" $O/walk_ab_$v.log
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max -d $O/pmc_$v -o run --output-format csv \
    -- python scripts/spmm_walk_ab.py 2 arxiv_gcn > $O/pmc_$v.log 2>&1 || exit $?
done
exit 0
