#!/bin/bash
# Interleaved A/B of environment settings for one library: bench lines per
# setting and config, repeated; prints ms/step and the assign kernel's own
# duration.   ab_env.sh "NAME=VAL;NAME2=VAL ..." [configs "cfg:semantics ..."]
# (settings separated by spaces; "-" = no extra variable)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abenv}
mkdir -p $O
CFGS="${2:-arxiv_gcn:update}"
for rep in 1 2; do
  for cs in $CFGS; do
    cfg=${cs%%:*}; sem=${cs#*:}
    i=0
    for setting in $1; do
      i=$((i+1))
      envs=""
      [ "$setting" != "-" ] && envs=$(echo "$setting" | tr ';' ' ')
      f=$O/ab${i}_${cfg}_${sem}_$rep
      env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --config $cfg \
        --semantics $sem > $f.json 2> $f.err || exit 1
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); k=d['kernels']['vq_assign']; print('$rep $cfg $sem [$setting]', 'ms/step %.4f'%d['ms_per_step'], 'assign us %.1f'%(k['ms_per_launch']*1e3))"
    done
  done
done
