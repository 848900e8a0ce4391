#!/bin/bash
# Round 6: the whole aggregation on a side stream beside the VQ update
# (--overlap-whole) for the configs whose aggregation is not the codebook
# source: arxiv_gat (gather + fused GAT aggregation) and ppi_sage (gather +
# two-source SpMM), against their serial step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06m
mkdir -p $O
run() {
  local name=$1; shift
  timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err \
    || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],4), d['config']['schedule'])"
}
for r in 1 2; do
  for cfg in arxiv_gat ppi_sage; do
    run ${cfg}_serial_$r --config $cfg
    run ${cfg}_whole_$r --config $cfg --overlap-whole
  done
done
