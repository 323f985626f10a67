#!/bin/bash
# One GPU session without the full test suite: selected tests (pytest -k), the bench line,
# rocprofv3 kernel stats, PMC FETCH/WRITE, and the C4 stage-phase profile.
# Usage (via gpurun): bash tools/gpu_bench.sh <tag> [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-bench}
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$2" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$2" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head -20; tail -30 $O/pytest.log; exit 1; }
  grep -E "passed|failed" $O/pytest.log | tail -1
fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-c4 > $O/kt.log 2>&1 || { echo "rocprof kt failed"; tail -30 $O/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -30 $O/pmc_write.log; exit 1; }
timeout -k 10 300 python -u tools/stage_profile.py dg316L3 > $O/stage_profile_dg316L3.txt 2>&1 || { echo "stage profile failed"; tail -20 $O/stage_profile_dg316L3.txt; exit 1; }
head -12 $O/stage_profile_dg316L3.txt
echo "bench $TAG done"
