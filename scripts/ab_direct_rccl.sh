#!/bin/bash
# One-rank RCCL rehearsal of the bench step: direct RCCL calls (default)
# against torch.distributed's process group (VQGNN_DIRECT_RCCL=0), eager and
# graph-captured, beside the plain one-GPU step.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/direct; mkdir -p $O
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 > $O/plain.json 2>$O/plain.err || exit 1
  python3 -c "import json; d=json.loads([l for l in open('$O/plain.json') if l.startswith('{')][-1]); print('plain', 'ms/step %.4f'%d['ms_per_step'])"
  for d in 1 0; do for g in "" "--graph"; do
    VQGNN_DIRECT_RCCL=$d timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 \
      --master-addr 127.0.0.1 --master-port $((29650 + rep)) bench.py --no-cpu-baseline --steps 30 --warmup 5 \
      --force-comm $g > $O/comm.json 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('$O/comm.json') if l.startswith('{')][-1]); print('comm direct=$d $g', 'ms/step %.4f'%d['ms_per_step'], 'host %.4f'%d.get('host_issue_ms_per_step',0))"
  done; done
done
