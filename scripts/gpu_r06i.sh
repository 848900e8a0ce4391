#!/bin/bash
# Round 6: parity of the library with the static single-chunk assign and the
# split walk / fix-up entries (VQ, defer, dist incl. the side-stream code
# landing), then the overlapped step in the one-rank RCCL rehearsal.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_vq.py tests/test_gpu_configs.py tests/test_gpu_defer.py \
  tests/test_gpu_dist.py -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $O/test.log 2>&1 \
  || { tail -40 $O/test.log; exit 1; }
grep -E "passed|failed" $O/test.log | tail -1
for ov in on off; do
  timeout -k 10 200 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --gpus 1 --force-comm --overlap $ov --steps 20 --warmup 5 --no-cpu-baseline \
    > $O/rehearsal_$ov.json 2> $O/rehearsal_$ov.err || { echo "FAIL rehearsal $ov"; tail -20 $O/rehearsal_$ov.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/rehearsal_$ov.json').read().strip().splitlines()[-1]); print('rehearsal $ov', round(d['ms_per_step'],4), d['config']['schedule'])"
done
