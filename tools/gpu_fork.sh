#!/bin/bash
# Glue-fork A/B (HNUMO_SCHED_DBG=4: one stream) + a step timeline.  Usage (via gpurun): bash tools/gpu_fork.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for c in dg25L3 bump16; do
  AB_REPS=3 timeout -k 10 300 python3 -u tools/ab_env.py $c "" "HNUMO_SCHED_DBG=4" > $O/abenv_$c.log 2>&1 || { echo "ab_env $c failed"; tail -20 $O/abenv_$c.log; exit 1; }
  grep -v amdgpu.ids $O/abenv_$c.log
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/kt -o run --output-format csv -- python3 tools/ab_stage.py dg25L3:persist > $O/kt.log 2>&1 || { echo "kt failed"; tail -20 $O/kt.log; exit 1; }
f=$(find $O/kt -name '*kernel_trace.csv' | head -1)
python3 tools/step_timeline.py $f 1 > $O/timeline.txt && cat $O/timeline.txt
echo "fork done"
