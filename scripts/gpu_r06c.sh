#!/bin/bash
# Overlap study: the codebook-source aggregation on a
# side stream beside BN statistics + assign, with and without workgroup
# shapes that let both kernels sit on one CU.  Interleaved, two rounds.
set -o pipefail
mkdir -p gpurun_out/r06c
O=gpurun_out/r06c
run() {   # name, env..., then bench flags after --
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env "${envs[@]}" timeout -k 10 120 python -u bench.py --steps 40 --warmup 10 --no-cpu-baseline "$@" \
    > $O/$name.json 2> $O/$name.err || { echo "FAIL $name"; tail -5 $O/$name.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],4))"
}
L=VQGNN_LIB=vq-gnn_amd/lib/ab_ovl.so
CO="VQGNN_ASG_TARGET=256 VQGNN_ASG_WAVES=8 VQGNN_CB_G=16 VQGNN_CB_NT=512 VQGNN_CB_WGS=128"
for r in 1 2; do
  run base_sep_$r X=1 -- --separate-finalize
  run ovl_sep_serial_$r $L -- --separate-finalize
  run ovl_default_$r $L -- --overlap
  run ovl_coshape_$r $L $CO -- --overlap
  run ser_coshape_$r $L $CO -- --separate-finalize
  run ovl_cbonly_$r $L VQGNN_CB_G=16 VQGNN_CB_NT=512 VQGNN_CB_WGS=128 -- --overlap
  run ovl_cb16_$r $L VQGNN_CB_G=16 VQGNN_CB_NT=512 -- --overlap
  run ovl_asg256_$r $L VQGNN_ASG_TARGET=256 VQGNN_ASG_WAVES=8 VQGNN_CB_G=16 VQGNN_CB_NT=512 -- --overlap
done
