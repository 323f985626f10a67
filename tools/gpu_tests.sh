#!/bin/bash
# GPU session: parity tests then one bench line.  Usage (via gpurun): bash tools/gpu_tests.sh <tag> [pytest args]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r02}
shift
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread "$@" > $O/pytest_gpu.log 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/pytest_gpu.log | tail -80
[ $rc -eq 0 ] || { echo "pytest rc=$rc"; tail -40 $O/pytest_gpu.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
