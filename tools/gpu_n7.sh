#!/bin/bash
# N=7 slim-arena check: parity subset, then A/B stage timing against a reference build.
# Usage (via gpurun): bash tools/gpu_n7.sh <tag> <ref.so>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "n7 or N7 or persistent or golden or bitwise" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python -u tools/ab_stage.py dg25N7L3:persist dg25N7L3:stage dg25L3:persist > $O/ab_new.log 2>&1 || { echo "ab new failed"; tail -20 $O/ab_new.log; exit 1; }
cat $O/ab_new.log
HNUMO_LIB=$2 timeout -k 10 300 python -u tools/ab_stage.py dg25N7L3:persist dg25N7L3:stage > $O/ab_ref.log 2>&1 || { echo "ab ref failed"; tail -20 $O/ab_ref.log; exit 1; }
cat $O/ab_ref.log
