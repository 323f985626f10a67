#!/bin/bash
# LDS / VALU counters of the stage kernels of several engine builds at one configuration, one
# --pmc pass per build (kernel-trace only).  Usage (via gpurun):
#   bash tools/gpu_pmc_ab.sh <tag> <cfg> "<lib1.so ...|default>"
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/$1
CFG=$2
mkdir -p $O
SET="SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64"
for lib in $3; do
  n=$(basename $lib .so)
  d=$O/pmc_${CFG}_$n
  if [ "$lib" = default ]; then L=""; else L=$lib; fi
  HNUMO_LIB=$L timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $SET -d $d -o run --output-format csv -- python3 tools/stage_only.py $CFG 1 > $d.log 2>&1 || { echo "pmc $n failed"; tail -5 $d.log; exit 1; }
  python3 - "$d" "$n" <<'PY'
import csv, glob, collections, sys
agg = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "btp_s" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
with open(sys.argv[1] + "/summary.txt", "w") as fh:
    for k, v in sorted(agg.items()):
        line = f"{sys.argv[2]:10s} {k:24s} {sum(v)/len(v):16.1f}  (mean per dispatch, n={len(v)})"
        print(line)
        fh.write(line + "\n")
PY
done
