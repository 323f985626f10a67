#!/bin/bash
# Per-kernel glue times of the dg25L3 step for engine builds: rocprofv3 kernel stats of
# tools/ab_stage.py under each library.  Usage (via gpurun): bash tools/gpu_glue.sh <tag> <libs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for lib in "$@"; do
  n=$(basename $lib .so)
  if [ "$lib" = default ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run --output-format csv -- python3 tools/ab_stage.py dg25L3:persist > $O/kt_$n.log 2>&1 || { echo "kt $n failed"; tail -20 $O/kt_$n.log; exit 1; }
  else
    HNUMO_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$n -o run --output-format csv -- python3 tools/ab_stage.py dg25L3:persist > $O/kt_$n.log 2>&1 || { echo "kt $n failed"; tail -20 $O/kt_$n.log; exit 1; }
  fi
  tail -1 $O/kt_$n.log
done
echo "glue $O done"
