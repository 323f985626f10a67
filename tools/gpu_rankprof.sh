#!/bin/bash
# Kernel traces of the C4 per-rank cost variants (tools/c4_rank_cost.py): the single-rank block
# and the self-neighbour RCCL rank, one rocprofv3 --kernel-trace --stats run each.
# Usage (via gpurun): bash tools/gpu_rankprof.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-rankprof}
mkdir -p $O
for v in block rccl; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o run --output-format csv -- python3 tools/c4_rank_cost.py --variants $v --steps 2 > $O/kt_$v.log 2>&1 || { echo "kt $v failed"; tail -20 $O/kt_$v.log; exit 1; }
  grep variant $O/kt_$v.log | head -2
done
echo "rankprof done"
