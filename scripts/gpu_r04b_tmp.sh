cd $GRAFT_REPO_ROOT; O=gpurun_out/r04c; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm_hot.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > $O/pytest_hot.log 2>&1; rc=$?
echo "hot tests rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest_hot.log | tail -5
if [ $rc -gt 1 ]; then exit $rc; fi
HOT_DBG="4 1 2 3 7" timeout -k 10 300 python -u scripts/bench_spmm_hot.py arxiv_gcn > $O/bench_hot.log 2>&1; rc=$?
echo "bench_hot rc=$rc"; cat $O/bench_hot.log | grep -v amdgpu.ids
if [ $rc -gt 1 ]; then exit $rc; fi
export TMPDIR=/tmp
VQGNN_SPMM_PLAN=hot TAG=r04c_hot TARGET=spmm PMC_LIST="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD
SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_SMEM SQ_ACTIVE_INST_VALU SQ_INSTS_VMEM_WR
TCC_HIT TCC_MISS GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE" bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1; rc=$?
echo "pmc rc=$rc"; python scripts/pmc_summary.py gpurun_out/pmc_r04c_hot > $O/pmc_summary.txt; grep -A 22 "spmm_hot_kernel\|spmm_task_kernel" $O/pmc_summary.txt | head -60
exit $rc
