cd $GRAFT_REPO_ROOT
O=gpurun_out/graph; mkdir -p $O
for rep in 1 2; do
for g in "" "--graph"; do
timeout -k 10 200 python bench.py --no-cpu-baseline --steps 30 --warmup 5 $g > $O/plain.json 2>$O/plain.err || { tail -3 $O/plain.err; exit 1; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=1 --master-addr 127.0.0.1 --master-port $((29600+rep)) bench.py --no-cpu-baseline --steps 30 --warmup 5 --force-comm $g > $O/comm.json 2>$O/comm.err || { tail -5 $O/comm.err; exit 1; }
for v in plain comm; do python3 -c "import json; d=json.loads([l for l in open('$O/$v.json') if l.startswith('{')][-1]); print('$v graph=$g', 'ms/step %.4f'%d['ms_per_step'], 'host %.4f'%d.get('host_issue_ms_per_step',0))"; done
done; done
