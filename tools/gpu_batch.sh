#!/bin/bash
# One GPU session of diagnostics: optional full GPU suite, stage-phase profiles, a dbg sweep and
# an A/B of engine builds.  Usage (via gpurun):
#   bash tools/gpu_batch.sh <tag> <tests:0|1> "<profile cfgs>" "<dbg cfg> <dbg values...>" "<libs>" <ab configs...>
# (empty strings skip a part)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
TESTS=$2
PROF=$3
DBG=$4
LIBS=$5
shift 5
mkdir -p $O
if [ "$TESTS" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
  tail -1 $O/pytest_gpu.log
fi
for c in $PROF; do
  timeout -k 10 300 python -u tools/stage_profile.py $c > $O/stage_profile_$c.txt 2>&1 || { echo "stage profile $c failed"; tail -20 $O/stage_profile_$c.txt; exit 1; }
  head -14 $O/stage_profile_$c.txt
done
if [ -n "$DBG" ]; then
  timeout -k 10 300 python -u tools/dbg_sweep.py $DBG > $O/dbg_sweep.txt 2>&1 || { echo "dbg sweep failed"; tail -20 $O/dbg_sweep.txt; exit 1; }
  cat $O/dbg_sweep.txt
fi
for lib in $LIBS; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then
    timeout -k 10 300 python -u tools/ab_stage.py "$@" > $O/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -20 $O/ab_$n.log; exit 1; }
  else
    HNUMO_LIB=$lib timeout -k 10 300 python -u tools/ab_stage.py "$@" > $O/ab_$n.log 2>&1 || { echo "ab $n failed"; tail -20 $O/ab_$n.log; exit 1; }
  fi
  cat $O/ab_$n.log
done
echo "batch $1 done"
