cd $GRAFT_REPO_ROOT; O=gpurun_out/r04d; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_hot.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_hot.log 2>&1; rc=$?
echo "hot tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_hot.log | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
HOT_SETS="8192,0 8192,256 4096,256 16384,256 4096,128 2048,256 16384,1024" HOT_DBG="1" timeout -k 10 300 python -u scripts/bench_spmm_hot.py arxiv_gcn > $O/bench_hot.log 2>&1; rc=$?
echo "bench_hot rc=$rc"; cat $O/bench_hot.log | grep -v amdgpu.ids
if [ $rc -gt 1 ]; then exit $rc; fi
for rep in 1 2; do for w in 0 10; do for sem in update feature_update; do
VQGNN_ASG_WAVES=$w timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --semantics $sem > $O/asg_${w}_${sem}_$rep.log 2>&1; rc=$?
if [ $rc -gt 1 ]; then echo "bench rc=$rc"; exit $rc; fi
python - $O/asg_${w}_${sem}_$rep.log $w $sem <<'PY'
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')]
d=json.loads(l[-1]); k=d['kernels']
print(f"waves={sys.argv[2]} {sys.argv[3]:15s} step {d['ms_per_step']*1e3:.1f} us  assign {k['vq_assign']['ms_per_launch']*1e3:.1f} us  spmm {k['spmm_ms']*1e3:.1f} us")
PY
done; done; done
exit 0
