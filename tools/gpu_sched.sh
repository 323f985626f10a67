#!/bin/bash
# The two-stream schedule of a processor-face rank at C4/8 size on one GPU: parity of the
# multi-rank tests, the per-rank cost (tools/c4_rank_cost.py) and its kernel trace, and timing
# experiments (HNUMO_SCHED_DBG; wrong results, timing only).  Usage: bash tools/gpu_sched.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-sched}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rccl_self_gpu.py tests/test_facehalo_gpu.py tests/test_multirank_gpu.py -m gpu -v --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/c4_rank_cost.py --variants block,rccl,rccl_g --steps 3 > $O/cost.log 2>&1 || { echo "cost failed"; tail -20 $O/cost.log; exit 1; }
grep variant $O/cost.log | head -3
HNUMO_SCHED_DBG=2 timeout -k 10 300 python -u tools/c4_rank_cost.py --variants rccl,rccl_g --steps 3 > $O/cost_dbg1.log 2>&1 || { echo "cost dbg1 failed"; tail -20 $O/cost_dbg1.log; exit 1; }
grep variant $O/cost_dbg1.log | head -2
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt_rccl -o run --output-format csv -- python3 tools/c4_rank_cost.py --variants rccl --steps 2 > $O/kt_rccl.log 2>&1 || { echo "kt failed"; tail -20 $O/kt_rccl.log; exit 1; }
echo "sched done"
