#!/bin/bash
# Kernel trace of the one-rank RCCL rehearsal (bench --force-comm).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof_comm}
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -T -d $O -o run --output-format csv -- \
  python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --no-cpu-baseline --steps 20 --warmup 5 --config ${CFG:-arxiv_gcn} --force-comm \
  > $O/bench.log 2>&1
rc=$?; echo "rc=$rc"; grep '^{' $O/bench.log | cut -c1-200; exit $rc
