#!/bin/bash
# Stage-arena A/B: parity of every arena, then C4 per-stage timing per arena (current build) and
# the reference build.  Usage (via gpurun): bash tools/gpu_nb.sh <tag> <ref.so>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
REF=$2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "stage_arenas or c4 or golden" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for nb in 4 5; do
  HNUMO_STAGE_NB=$nb timeout -k 10 300 python -u tools/ab_stage.py dg316L3:stage dg25L3:stage > $O/ab_nb$nb.log 2>&1 || { echo "ab nb$nb failed"; tail -20 $O/ab_nb$nb.log; exit 1; }
  cat $O/ab_nb$nb.log
done
HNUMO_LIB=$REF timeout -k 10 300 python -u tools/ab_stage.py dg316L3:stage dg25L3:stage > $O/ab_ref.log 2>&1 || { echo "ab ref failed"; tail -20 $O/ab_ref.log; exit 1; }
cat $O/ab_ref.log
