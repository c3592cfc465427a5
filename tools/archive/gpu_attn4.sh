set -o pipefail
mkdir -p gpurun_out/attn4
O=gpurun_out/attn4
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "attention" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 120 python -u tools/attn_one.py 20 > $O/timing.log 2>&1 && cat $O/timing.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM --output-format csv -d $GRAFT_REPO_ROOT/$O/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/attn_one.py 3 > $GRAFT_REPO_ROOT/$O/p2.log 2>&1
echo "pmc rc=$?"
