#!/bin/bash
# Parity subset, then A/B step/stage timing of the current build against a reference build.
# Usage (via gpurun): bash tools/gpu_ab.sh <tag> <ref.so> <pytest -k expr> <ab_stage configs...>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
REF=$2
K=$3
shift 3
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_stage.py "$@" > $O/ab_new.log 2>&1 || { echo "ab new failed"; tail -20 $O/ab_new.log; exit 1; }
HNUMO_LIB=$REF timeout -k 10 300 python -u tools/ab_stage.py "$@" > $O/ab_ref.log 2>&1 || { echo "ab ref failed"; tail -20 $O/ab_ref.log; exit 1; }
cat $O/ab_new.log $O/ab_ref.log
