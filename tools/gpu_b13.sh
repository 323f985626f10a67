set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/b13
mkdir -p $O
AB_REPS=2 timeout -k 10 300 python -u tools/ab_env.py dg25L3:persist "" "HNUMO_PLACE=0" > $O/ab_place_dg25.log 2>&1 || { echo fail1; tail $O/ab_place_dg25.log; exit 1; }
cat $O/ab_place_dg25.log
AB_REPS=2 timeout -k 10 300 python -u tools/ab_env.py dg25N7L3:persist "" "HNUMO_PLACE=0" > $O/ab_place_n7.log 2>&1 || { echo fail2; tail $O/ab_place_n7.log; exit 1; }
cat $O/ab_place_n7.log
HNUMO_LIB=scratch_libs/u3t.so timeout -k 10 300 python -u tools/ab_stage.py dg25N7L3:persist > $O/ab_u3t.log 2>&1 || { echo fail3; exit 1; }
cat $O/ab_u3t.log
timeout -k 10 300 python -u tools/stage_profile.py dg25L3 > $O/stage_profile_dg25L3.txt 2>&1 || { echo fail4; exit 1; }
grep -E "CUs with|trace wait per|stage avg" $O/stage_profile_dg25L3.txt
echo done
