#!/bin/bash
# Persistent-launch residency: the fallback tests, the estimate-vs-dispatcher sweep, the parity
# subset and a short bench.  Usage (via gpurun): bash tools/gpu_persist.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_persistent_residency_gpu.py -v --timeout 120 --timeout-method thread > $O/pytest_persist.log 2>&1 || { echo "persist tests failed"; tail -40 $O/pytest_persist.log; exit 1; }
grep -E "PASSED|FAILED" $O/pytest_persist.log
timeout -k 10 300 python -u tools/residency_sweep.py dg25L3 0 2560 256 > $O/sweep_dg25L3.txt 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_dg25L3.txt; exit 1; }
cat $O/sweep_dg25L3.txt
timeout -k 10 300 python -u tools/residency_sweep.py dg25N7L3 0 2560 256 > $O/sweep_dg25N7L3.txt 2>&1 || { echo "sweep failed"; tail -20 $O/sweep_dg25N7L3.txt; exit 1; }
cat $O/sweep_dg25N7L3.txt
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "bitwise or golden or facehalo" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
