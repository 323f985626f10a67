#!/bin/bash
# Quick GPU check: the bitwise parity subset, then kernel stats of a short bench.
# Usage (via gpurun): bash tools/gpu_quick.sh <tag> [pytest -k expr]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-quick}
K=${2:-"bitwise or golden or facehalo or partition"}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -k "$K" > $O/pytest.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" $O/pytest.log | head; tail -20 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --no-cpu-baseline --no-c4 --steps 10 > $O/bench.json 2> $O/kt.log || { echo "rocprof failed"; tail -20 $O/kt.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, json, sys
b = [l for l in open(sys.argv[1] + "/bench.json") if l.startswith("{")]
if b:
    d = json.loads(b[-1]); print("bench", d["value"], "EU/s", d["ms_per_step"], "ms/step")
f = glob.glob(sys.argv[1] + "/kt/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows[:14]:
    print(f'{r["Name"][:60]:60s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1e3:9.2f} us {float(r["Percentage"]):6.2f}%')
PY
