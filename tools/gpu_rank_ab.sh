#!/bin/bash
# Per-GPU cost of the C4/8 rank (tools/c4_rank_cost.py, block and RCCL variants) for engine builds,
# 2 interleaved repetitions.  Usage (via gpurun): bash tools/gpu_rank_ab.sh <tag> <libs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for rep in 1 2; do
for lib in "$@"; do
  n=$(basename $lib .so)
  HNUMO_LIB=$lib timeout -k 10 300 python3 -u tools/c4_rank_cost.py --steps 3 --variants block,rccl --no-projection > $O/rank_${n}_$rep.log 2>&1 || { echo "rank $n failed"; tail -20 $O/rank_${n}_$rep.log; exit 1; }
  echo "== $n $rep"; grep '"variant"' $O/rank_${n}_$rep.log | cut -c1-160
done
done
echo "rank ab done"
