#!/bin/bash
# Parity of the current build (GPU suite) and A/B timing of engine builds (tools/ab_stage.py, state
# hashes: equal = same bits).  Usage (via gpurun): bash tools/gpu_ab2.sh <tag> "<configs>" <libs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
AB=$2
shift 2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
for lib in "$@"; do
  HNUMO_LIB=$lib timeout -k 10 300 python -u tools/ab_stage.py $AB > $O/ab_$(basename $lib .so)_$rep.log 2>&1 || { echo "ab $lib failed"; tail -20 $O/ab_$(basename $lib .so)_$rep.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$(basename $lib .so)_$rep.log
done
done
echo "ab2 done"
