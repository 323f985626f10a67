#!/bin/bash
# timing + phase/wait profile of each variant (current build and h-numo_amd/exp/*.so)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}; mkdir -p $O
for lib in h-numo_amd/libhnumo_engine.so h-numo_amd/exp/*.so; do
  b=$(basename $lib .so)
  HNUMO_LIB=$PWD/$lib timeout -k 10 60 python tools/stage_only.py dg25L3 4 > $O/t_$b.txt 2>&1 || { tail $O/t_$b.txt; exit 1; }
  HNUMO_LIB=$PWD/$lib timeout -k 10 60 python tools/stage_profile.py dg25L3 > $O/p_$b.txt 2>&1 || { tail $O/p_$b.txt; exit 1; }
  echo "== $b: $(cat $O/t_$b.txt)"; grep -A20 "persistent:" $O/p_$b.txt
done
