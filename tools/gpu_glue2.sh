#!/bin/bash
# Step timeline (kernel trace of tools/ab_stage.py dg25L3) and the baroclinic kernels' phase clocks
# (HNUMO_BCL_PROF build).  Usage (via gpurun): bash tools/gpu_glue2.sh <tag> <bclprof .so> [libs...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
P=$2
shift 2
mkdir -p $O
HNUMO_LIB=$P timeout -k 10 300 python3 -u tools/bcl_profile.py dg25L3 > $O/bcl_phase_profile_dg25L3.txt 2>&1 || { echo "bcl_profile failed"; tail -20 $O/bcl_phase_profile_dg25L3.txt; exit 1; }
grep -v amdgpu.ids $O/bcl_phase_profile_dg25L3.txt
for lib in h-numo_amd/libhnumo_engine.so "$@"; do
  n=$(basename $lib .so)
  HNUMO_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt_$n -o run --output-format csv -- python3 tools/ab_stage.py dg25L3:persist > $O/kt_$n.log 2>&1 || { echo "kt $n failed"; tail -20 $O/kt_$n.log; exit 1; }
  f=$(find $O/kt_$n -name '*kernel_trace.csv' | head -1)
  python3 tools/step_timeline.py $f 1 > $O/timeline_$n.txt && python3 tools/step_timeline.py $f 3 > $O/timeline3_$n.txt
  echo "== $n"; tail -14 $O/timeline3_$n.txt
done
echo "glue2 done"
