#!/bin/bash
# Iteration loop on the GPU box: bitwise parity tests, sub-cycle timing, phase clocks.
# Usage: bash tools/iter.sh <tag> [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-it}
mkdir -p $O
K=${2:-"bitwise or persistent or golden or subcycle or n7"}
timeout -k 10 300 python -u -m pytest tests/test_engine_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 100 python tools/stage_only.py dg25L3 4 > $O/time.txt 2>&1 || { cat $O/time.txt; exit 1; }
cat $O/time.txt
timeout -k 10 100 python tools/stage_profile.py dg25L3 > $O/prof.txt 2>&1 || { tail $O/prof.txt; exit 1; }
head -20 $O/prof.txt; tail -4 $O/prof.txt
