#!/bin/bash
# Stage timing of several engine builds on the same box.  Usage (via gpurun):
#   bash tools/gpu_multi_ab.sh <tag> "<lib1.so lib2.so ...|default>" <ab_stage configs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
LIBS=$2
shift 2
mkdir -p $O
for lib in $LIBS; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then
    timeout -k 10 300 python -u tools/ab_stage.py "$@" > $O/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -20 $O/ab_$n.log; exit 1; }
  else
    HNUMO_LIB=$lib timeout -k 10 300 python -u tools/ab_stage.py "$@" > $O/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -20 $O/ab_$n.log; exit 1; }
  fi
  cat $O/ab_$n.log
done
