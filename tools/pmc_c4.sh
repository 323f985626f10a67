#!/bin/bash
# Counters of the per-stage kernel at a configuration (default C4 = dg316L3): SQ instruction /
# stall counters and HBM FETCH/WRITE, one --pmc set per run (kernel-trace only).
# Usage (via gpurun): bash tools/pmc_c4.sh [cfg] [outdir]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CFG=${1:-dg316L3}
OUT=${2:-gpurun_out/pmc_$CFG}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_INST_ANY SQ_INSTS_SMEM" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/stage_only.py $CFG 1 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "btp_s" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(sys.argv[1] + "/summary.txt", "w") as fh:
    for k, v in sorted(agg.items()):
        line = f"{k:28s} {sum(v)/len(v):18.1f}  (mean per dispatch, n={len(v)})"
        print(line)
        fh.write(line + "\n")
PY
