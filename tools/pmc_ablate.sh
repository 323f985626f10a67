#!/bin/bash
# Instruction mix of the per-stage kernel with diagnostic phase switches (HNUMO_STAGE_DBG bits:
# 1 face lifts, 2 Laplacian, 4 volume sums, 32 time averages, 64 term tasks; with a
# -DHNUMO_DBG_EXTRA=1 build also 128 A2 interpolations, 256 B quad tasks, 512 B face tasks, 1024 B
# nodal tasks, 2048 E2 trace stores, 4096 the A record copies (only with 2048: the trace slots
# come from the records); counting only, they break the physics): SQ_INSTS_* per element-stage
# for each switch, one rocprofv3 run each.  DBGS overrides the list of switches.
# Usage (via gpurun): bash tools/pmc_ablate.sh <outdir> [cfg] [lib.so ...]
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=${1:-gpurun_out/ablate}
CFG=${2:-dg316L3}
shift 2
LIBS=${*:-default}
mkdir -p $OUT
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_FMA_F64"
for lib in $LIBS; do
  tag=$(basename $lib .so)
  for dbg in ${DBGS:-0 64 4 1 2 32 68}; do
    if [ "$lib" = default ]; then L=""; else L=$lib; fi
    HNUMO_LIB=$L HNUMO_EXPERIMENTS=1 HNUMO_STAGE_DBG=$dbg timeout -s KILL 180 rocprofv3 --kernel-trace --pmc $SQ -d $OUT/${tag}_d$dbg -o run --output-format csv -- python3 tools/stage_only.py $CFG 1 > $OUT/${tag}_d$dbg.log 2>&1 || { echo "pass $tag dbg $dbg failed"; tail -5 $OUT/${tag}_d$dbg.log; exit 1; }
  done
done
python3 - "$OUT" "$CFG" <<'PY'
import csv, glob, collections, sys, os
out, cfg = sys.argv[1], sys.argv[2]
E = {"dg316L3": 99856, "dg25L3": 625, "dg25N7L3": 625}[cfg]
rows = []
for d in sorted(glob.glob(out + "/*_d*/")):
    agg = collections.defaultdict(list)
    for f in glob.glob(d + "**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if "btp_stage_kernel" in r["Kernel_Name"]:
                agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    m = {k: sum(v) / len(v) / E for k, v in agg.items()}
    rows.append((os.path.basename(d.rstrip("/")), m))
keys = ["SQ_INSTS_VALU", "SQ_INSTS_VALU_INT32", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_SALU", "SQ_INSTS_LDS"]
with open(out + "/summary.txt", "w") as fh:
    hdr = f"{'run':24s}" + "".join(f"{k[9:]:>12s}" for k in keys)
    print(hdr); fh.write(hdr + "\n")
    for name, m in rows:
        line = f"{name:24s}" + "".join(f"{m.get(k, 0):12.1f}" for k in keys)
        print(line); fh.write(line + "\n")
PY
