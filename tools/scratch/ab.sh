#!/bin/bash
# A/B timing of sub-cycle variants: current build vs h-numo_amd/exp/*.so, coupled and with
# the trace waits skipped (dbg 16: wrong results, pure per-element work).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-ab}; mkdir -p $O
for lib in h-numo_amd/libhnumo_engine.so h-numo_amd/exp/*.so; do
  for dbg in ${DBGS:-0}; do
    r=$(HNUMO_LIB=$PWD/$lib HNUMO_STAGE_DBG=$dbg timeout -k 10 60 python tools/stage_only.py dg25L3 4 2>&1 | tail -1) || { echo "$lib $dbg failed: $r"; exit 1; }
    echo "$(basename $lib) dbg=$dbg: $r" | tee -a $O/ab.txt
  done
done
