#!/bin/bash
# Interleaved A/B of library variants (VQGNN_LIB) on one box for the assign
# kernel: bench lines per variant and config, repeated; prints ms/step and
# the assign kernel's own duration (hipExtLaunchKernel events).
#   ab_assign.sh "name ..." [configs: "cfg:semantics ..."]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${TAG:-ab}
mkdir -p $O
VARS="$1"
CFGS="${2:-arxiv_gcn:update}"
for rep in ${REPS:-1 2}; do
  for cs in $CFGS; do
    cfg=${cs%%:*}; sem=${cs#*:}
    for n in $VARS; do
      # a variant is "default", a library name (vq-gnn_amd/lib/ab_<name>.so) or
      # environment settings "K=V[+K=V...]" on the default library
      unset VQGNN_LIB; envs=""
      case $n in
        default) ;;
        *=*) envs=$(echo $n | tr '+' ' ') ;;
        *) export VQGNN_LIB=$PWD/vq-gnn_amd/lib/ab_$n.so ;;
      esac
      env $envs timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --config $cfg \
        --semantics $sem > $O/ab_${n}_${cfg}_${sem}_$rep.json 2> $O/ab_${n}_${cfg}_${sem}_$rep.err || exit 1
      python3 -c "import json; d=json.loads(open('$O/ab_${n}_${cfg}_${sem}_$rep.json').read().strip().splitlines()[-1]); k=d['kernels']['vq_assign']; print('$rep $cfg $sem $n', 'ms/step %.4f'%d['ms_per_step'], 'assign us %.1f'%(k['ms_per_launch']*1e3), 'frac %.3f'%k['frac'])"
    done
  done
done
