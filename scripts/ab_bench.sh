#!/bin/bash
# Interleaved A/B of bench.py variants on one box: bench lines per variant and
# config, repeated twice; prints ms/step, the assign kernel's own duration and
# the aggregation phase.
#   ab_bench.sh "name|ENV=V;ENV2=V|--flag --flag2 ..." ["cfg:semantics ..."]
# (a variant: name, then ';'-separated environment settings, then bench flags;
# either part may be empty; VQGNN_LIB=... selects a library build)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-abbench}
mkdir -p $O
CFGS="${2:-arxiv_gcn:update}"
IFS=$'\n' read -r -d '' -a VARS < <(echo "$1" | tr ' ' '\n' | sed 's/~/ /g' && printf '\0')
for rep in 1 2; do
  for cs in $CFGS; do
    cfg=${cs%%:*}; sem=${cs#*:}
    for v in "${VARS[@]}"; do
      name=$(echo "$v" | cut -d'|' -f1)
      envs=$(echo "$v" | cut -d'|' -f2 | tr ';' ' ')
      flags=$(echo "$v" | cut -d'|' -f3)
      f=$O/${name}_${cfg}_${sem}_$rep
      env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 \
        --config $cfg --semantics $sem $flags > $f.json 2> $f.err || exit 1
      python3 -c "import json; d=json.loads(open('$f.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$rep $cfg $sem $name', 'ms/step %.4f'%d['ms_per_step'], 'assign us %.1f'%(k['vq_assign']['ms_per_launch']*1e3), 'agg us %.1f'%(k['spmm_ms']*1e3), d['config'].get('aggregation'), '|', d['config'].get('order'))"
    done
  done
done
