#!/bin/bash
# Round-4 GPU session: GPU suite, bench line, A/B of engine builds, C4 instruction-mix ablation.
# Usage (via gpurun): bash tools/gpu_r04.sh <tag> [ab configs] [libs...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
AB=${2:-"dg316L3:stage dg25L3"}
shift 2
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest_gpu.log | head -20; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -30 $O/bench.err; exit 1; }
cat $O/bench.json
fi
for lib in "$@"; do
  HNUMO_LIB=$lib timeout -k 10 300 python -u tools/ab_stage.py $AB > $O/ab_$(basename $lib .so).log 2>&1 || { echo "ab $lib failed"; tail -20 $O/ab_$(basename $lib .so).log; exit 1; }
  cat $O/ab_$(basename $lib .so).log
done
echo "session $TAG done"
