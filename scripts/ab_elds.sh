cd $GRAFT_REPO_ROOT
for rep in 1 2; do for cfg in arxiv_gat arxiv_gcn; do for e in 1 0; do
VQGNN_FLT_ELDS=$e timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 --config $cfg > gpurun_out/abe.json 2>/dev/null || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/abe.json').read().strip().splitlines()[-1]); k=d['kernels']['vq_assign']; print('$cfg elds=$e', 'ms/step %.4f'%d['ms_per_step'], 'assign us %.1f'%(k['ms_per_launch']*1e3))"
done; done; done
