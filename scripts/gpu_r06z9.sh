#!/bin/bash
# (re-run on the final library of round 6, lib e4055e60: output under gpurun_out/r06z9)
# Round 6: the multi-rank bench path on the final tree -- the one-rank RCCL
# rehearsal (--force-comm) and two gloo ranks sharing the one GPU
# (VQGNN_BENCH_ONE_DEVICE=1) -- and bench.py --gpus 2 as the driver launches it
# is not possible on a one-GPU box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06z9
mkdir -p $O
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 1 --force-comm --steps 20 --warmup 5 --no-cpu-baseline \
  > $O/rccl1.json 2> $O/rccl1.err || { echo FAIL rccl1; tail -20 $O/rccl1.err; exit 1; }
grep -h '^{' $O/rccl1.json | cut -c1-260
VQGNN_BENCH_ONE_DEVICE=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 \
  --master-addr 127.0.0.1 --master-port 29532 bench.py --gpus 2 --backend gloo --steps 10 --warmup 3 \
  --no-cpu-baseline > $O/gloo2.json 2> $O/gloo2.err || { echo FAIL gloo2; tail -20 $O/gloo2.err; exit 1; }
grep -h '^{' $O/gloo2.json | cut -c1-260
