#!/bin/bash
# Diagnostics session: C4 per-rank cost (tools/c4_rank_cost.py), stage phase profiles, and the
# C4 instruction-mix ablation (tools/pmc_ablate.sh).  Usage (via gpurun): bash tools/gpu_diag.sh <tag>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/${1:-diag}
mkdir -p $O
[ -n "$SKIP_COST" ] || timeout -k 10 500 python -u tools/c4_rank_cost.py --steps 3 > $O/c4_rank_cost.log 2>&1 || { echo "rank cost failed"; tail -20 $O/c4_rank_cost.log; exit 1; }
[ -n "$SKIP_COST" ] || grep -v amdgpu.ids $O/c4_rank_cost.log
for cfg in ${PROFILE_CFGS-dg25L3 dg25N7L3 dg316L3}; do
  timeout -k 10 300 python -u tools/stage_profile.py $cfg > $O/stage_profile_$cfg.txt 2>&1 || { echo "profile $cfg failed"; tail -20 $O/stage_profile_$cfg.txt; exit 1; }
done
bash tools/pmc_ablate.sh $O/ablate dg316L3 ${ABLATE_LIB:-default}
