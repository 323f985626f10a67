#!/bin/bash
# SQ instruction/stall counters over the barotropic sub-cycle kernel (persistent path, or the
# per-stage kernel with HNUMO_PERSISTENT=0); separate --pmc runs, kernel-trace only.
# Usage: bash tools/pmc_sq.sh [cfg] [outdir]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
CFG=${1:-dg25L3}
OUT=${2:-gpurun_out/pmcsq}
mkdir -p $OUT
i=0
for set in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_WAIT_INST_ANY" \
           "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_THREAD_CYCLES_VALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE GRBM_COUNT"; do
  timeout -k 10 180 rocprofv3 --kernel-trace --pmc $set -d $OUT/p$i -o run --output-format csv -- python3 tools/stage_only.py $CFG 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  i=$((i+1))
done
python3 - "$OUT" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/p*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "btp_s" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
