#!/bin/bash
# Roofline evidence for the three single-GPU BASELINE configs (dg25L3 = configs[1], dg25N7L3 = C3,
# dg316L3 = C4): per config one rocprofv3 --kernel-trace --stats run of bench.py, the FETCH_SIZE and
# WRITE_SIZE passes, and two SQ instruction-mix passes; each pass its own run.
# Usage (via gpurun): bash tools/gpu_profiles.sh <tag> [configs...]
# Then, here: python tools/profile_summary.py <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:-r04}
shift
CFGS=${*:-"dg25L3 dg25N7L3 dg316L3"}
O=gpurun_out/$TAG
mkdir -p $O
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64"
SQ2="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_BUSY_CYCLES"
for cfg in $CFGS; do
  case $cfg in
    dg316L3|lake200) S=3; W=1 ;;
    dg25N7L3) S=10; W=2 ;;
    *) S=20; W=3 ;;
  esac
  B="python3 bench.py --config $cfg --no-cpu-baseline --no-c4"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$cfg -o run --output-format csv -- $B --steps $S --warmup $W > $O/kt_$cfg.log 2>&1 || { echo "kt $cfg failed"; tail -20 $O/kt_$cfg.log; exit 1; }
  tail -1 $O/kt_$cfg.log
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $c -d $O/pmc_${c}_$cfg -o run --output-format csv -- $B --steps 2 --warmup 1 > $O/pmc_${c}_$cfg.log 2>&1 || { echo "pmc $c $cfg failed"; tail -20 $O/pmc_${c}_$cfg.log; exit 1; }
  done
  if true; then
    i=1
    for set in "$SQ1" "$SQ2"; do
      timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $set -d $O/pmc_sq${i}_$cfg -o run --output-format csv -- $B --steps 2 --warmup 1 > $O/pmc_sq${i}_$cfg.log 2>&1 || { echo "pmc sq$i $cfg failed"; tail -20 $O/pmc_sq${i}_$cfg.log; exit 1; }
      i=$((i+1))
    done
  fi
  echo "$cfg done"
done
echo "profiles $TAG done"
