#!/bin/bash
# Phase clocks of the v0 kernel at low load (bump10: 100 elements, < 1 per CU) vs dg25L3.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}; mkdir -p $O
for cfg in bump10 dg25L3; do
  HNUMO_LIB=$PWD/h-numo_amd/exp/libhnumo_engine_v0.so timeout -k 10 60 python tools/stage_profile.py $cfg > $O/prof_$cfg.txt 2>&1 || { tail $O/prof_$cfg.txt; exit 1; }
  HNUMO_PERSISTENT=0 HNUMO_LIB=$PWD/h-numo_amd/exp/libhnumo_engine_v0.so timeout -k 10 60 python tools/stage_profile.py $cfg > $O/profnp_$cfg.txt 2>&1 || { tail $O/profnp_$cfg.txt; exit 1; }
done
for f in $O/prof*.txt; do echo "== $f"; head -18 $f; tail -3 $f; done
