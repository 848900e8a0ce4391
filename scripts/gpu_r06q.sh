#!/bin/bash
# Round 6: the arxiv assign with 16-wave workgroups (one per CU) against the
# default 8-wave pair (ab_exp.so, VQGNN_ASG_WAVES), interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r06q
mkdir -p $O
X=$PWD/vq-gnn_amd/lib/ab_exp.so
for r in 1 2 3; do
  for w in 8 16; do
    for sem in update feature_update; do
      VQGNN_LIB=$X VQGNN_ASG_WAVES=$w timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 \
        --semantics $sem > $O/w${w}_${sem}_$r.json 2> $O/w${w}_${sem}_$r.err || { tail -5 $O/w${w}_${sem}_$r.err; exit 1; }
      python3 -c "import json; d=json.loads(open('$O/w${w}_${sem}_$r.json').read().strip().splitlines()[-1]); k=d['kernels']['vq_assign']; print('$r waves=$w $sem', 'ms/step %.4f'%d['ms_per_step'], 'assign us %.1f'%(k['ms_per_launch']*1e3))"
    done
  done
done
