#!/bin/bash
# One box, everything pending: GPU suite on the current build, A/B of engine builds, C4 per-rank
# cost, stage phase profiles, C4 instruction-mix ablation.
# Usage (via gpurun): bash tools/gpu_r04f.sh <tag> "<ab configs>" <libs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=$1
AB=$2
shift 2
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for lib in "$@"; do
  HNUMO_LIB=$lib timeout -k 10 300 python -u tools/ab_stage.py $AB > $O/ab_$(basename $lib .so).log 2>&1 || { echo "ab $lib failed"; tail -20 $O/ab_$(basename $lib .so).log; exit 1; }
  grep -v amdgpu.ids $O/ab_$(basename $lib .so).log
done
bash tools/gpu_diag.sh $TAG/diag
echo "session $TAG done"
