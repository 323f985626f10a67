#!/bin/bash
# Glue A/B: bitwise + step time (tools/ab_stage.py) and the element kernels' phase clocks
# (HNUMO_BCL_PROF builds) for pairs <lib> <prof lib>.  Usage (via gpurun):
#   bash tools/gpu_glue3.sh <tag> "<configs>" <lib1> <prof1> [<lib2> <prof2> ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
AB=$2
shift 2
mkdir -p $O
args=("$@")
for ((i = 0; i < ${#args[@]}; i += 2)); do
  lib=${args[i]}; prof=${args[i+1]}; n=$(basename $lib .so)
  HNUMO_LIB=$prof timeout -k 10 300 python3 -u tools/bcl_profile.py dg25L3 > $O/bcl_$n.txt 2>&1 || { echo "bcl_profile $n failed"; tail -20 $O/bcl_$n.txt; exit 1; }
  echo "== $n"; grep -v amdgpu.ids $O/bcl_$n.txt
done
for rep in 1 2; do
for ((i = 0; i < ${#args[@]}; i += 2)); do
  lib=${args[i]}; n=$(basename $lib .so)
  HNUMO_LIB=$lib timeout -k 10 300 python3 -u tools/ab_stage.py $AB > $O/ab_${n}_$rep.log 2>&1 || { echo "ab $n failed"; tail -20 $O/ab_${n}_$rep.log; exit 1; }
  grep -v amdgpu.ids $O/ab_${n}_$rep.log
done
done
echo "glue3 done"
