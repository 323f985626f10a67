#!/bin/bash
# Round-3 GPU session: the full GPU suite, the bench line, rocprofv3 kernel stats and the PMC
# FETCH/WRITE passes of the dg25L3 run.  Usage (via gpurun): bash tools/gpu_round3.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r03}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-c4 > $O/kt.log 2>&1 || { echo "rocprof kt failed"; tail -30 $O/kt.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; tail -30 $O/pmc_fetch.log; exit 1; }
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $O/pmc_write -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-c4 > $O/pmc_write.log 2>&1 || { echo "pmc write failed"; tail -30 $O/pmc_write.log; exit 1; }
echo "round $TAG done"
