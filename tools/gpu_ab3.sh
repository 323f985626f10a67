#!/bin/bash
# A/B timing only (no suite): tools/ab_stage.py over the given builds, 3 interleaved repetitions.
# Usage (via gpurun): bash tools/gpu_ab3.sh <tag> "<configs>" <libs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
AB=$2
shift 2
mkdir -p $O
for rep in 1 2 3; do
for lib in "$@"; do
  HNUMO_LIB=$lib timeout -k 10 300 python -u tools/ab_stage.py $AB > $O/ab_$(basename $lib .so)_$rep.log 2>&1 || { echo "ab $lib failed"; tail -20 $O/ab_$(basename $lib .so)_$rep.log; exit 1; }
  grep -v amdgpu.ids $O/ab_$(basename $lib .so)_$rep.log
done
done
echo "ab3 done"
