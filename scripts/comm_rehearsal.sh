#!/bin/bash
# Per-rank cost of the multi-GPU exchange machinery: the default bench
# against a one-rank RCCL world with every collective live (--force-comm).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-comm}
mkdir -p $O
for cfg in ${CFGS:-arxiv_gcn}; do for rep in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --config $cfg > $O/plain_$cfg.json 2>$O/plain.err || exit 1
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
    --master-port $((29500 + rep)) bench.py --no-cpu-baseline --steps 30 --warmup 5 --config $cfg --force-comm \
    > $O/comm_$cfg.json 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
  for v in plain comm; do
    python3 -c "import json; d=json.loads([l for l in open('$O/${v}_$cfg.json') if l.startswith('{')][-1]); print('$cfg $v', 'ms/step %.4f'%d['ms_per_step'])"
  done
done; done
