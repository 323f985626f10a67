#!/bin/bash
# One parameterised GPU session (via gpurun): the named steps in order, each under its own time
# limit, stopping at the first failure.  Output under gpurun_out/<tag>/.
#
#   bash tools/gpu_session.sh <tag> <step> [<step> ...]
#
# steps:
#   tests        pytest -m gpu (the whole GPU suite)
#   test:<expr>  pytest -m gpu -k <expr>
#   smoke        __graft_entry__.smoke()
#   bench        the default bench line (N=1: dg25L3 + C4 + C3 + CPU baselines)
#   benchq       the bench line without the CPU baselines
#   emu8         bench.py --emulate 8:1 (C4 rank 1 of 8) under torch.distributed.run, one process
#   emu4lake     bench.py --emulate 4:1 --config lake200 (C5 rank 1 of 4) the same way
#   nb56         tools/ab_env.py: C4 per-stage kernel, LEAN arena for 5 vs 6 workgroups per CU
#   sprof:<cfg>  tools/stage_profile.py with the diagnostics build diag/libhnumo_diag.so (phase clocks)
#   bclprof:<cfg>  tools/bcl_profile.py with the diagnostics build (element kernels' phase clocks)
#   abbd:<cfg[:stage]>:<KNOB>:<v1>/<v2>  tools/ab_breakdown.py (per-kernel step breakdown per value)
#   abbdl:<lib>:<cfg>  the same for a build (HNUMO_LIB)
#   abl:<lib>:<cfgs>  tools/ab_stage.py with HNUMO_LIB=<lib> (A/B of builds)
#   emu:W:R:cfg:order[:warmup:steps]  bench.py --emulate W:R --config cfg --order order
#   rank         tools/c4_rank_cost.py (C4/8 rank 1 variants)
#   rankprof     rocprofv3 kernel trace of tools/c4_rank_cost.py (block, rccl)
#   profiles     tools/gpu_profiles.sh <tag> (kernel trace + FETCH/WRITE + SQ passes)
#   prof:<cfg>   tools/gpu_profiles.sh <tag> <cfg>
#   ab:<args>    tools/ab_stage.py <args, commas for spaces>
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
TAG=${1:?tag}
shift
O=gpurun_out/$TAG
mkdir -p $O
fail() { echo "step $1 failed (rc $2)"; tail -30 "$3"; exit 1; }
TR="python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
for step in "$@"; do
  echo "[$(date +%T)] $step"
  case $step in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || fail "$step" $? $O/pytest_gpu.log
      tail -1 $O/pytest_gpu.log ;;
    test:*)
      k=${step#test:}
      timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$k" > $O/pytest_k.log 2>&1 || fail "$step" $? $O/pytest_k.log
      tail -1 $O/pytest_k.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || fail "$step" $? $O/smoke.log
      tail -1 $O/smoke.log ;;
    bench)
      timeout -k 10 900 python bench.py > $O/bench.json 2> $O/bench.err || fail "$step" $? $O/bench.err
      cat $O/bench.json ;;
    benchq)
      timeout -k 10 600 python bench.py --no-cpu-baseline > $O/benchq.json 2> $O/benchq.err || fail "$step" $? $O/benchq.err
      cat $O/benchq.json ;;
    emu8)
      timeout -k 10 600 $TR bench.py --emulate 8:1 > $O/emu8.json 2> $O/emu8.err || fail "$step" $? $O/emu8.err
      cat $O/emu8.json ;;
    emu4lake)
      timeout -k 10 600 $TR bench.py --emulate 4:1 --config lake200 > $O/emu4lake.json 2> $O/emu4lake.err || fail "$step" $? $O/emu4lake.err
      cat $O/emu4lake.json ;;
    lake1)
      timeout -k 10 600 python bench.py --config lake200 --no-cpu-baseline --steps 10 > $O/lake1.json 2> $O/lake1.err || fail "$step" $? $O/lake1.err
      cat $O/lake1.json ;;
    emu4lake2)
      timeout -k 10 600 $TR bench.py --emulate 4:1 --config lake200 --warmup 1 --steps 2 > $O/emu4lake2.json 2> $O/emu4lake2.err || fail "$step" $? $O/emu4lake2.err
      cat $O/emu4lake2.json ;;
    nb56)
      AB_REPS=2 timeout -k 10 600 python -u tools/ab_env.py dg316L3:stage HNUMO_STAGE_NB=5 HNUMO_STAGE_NB=6 > $O/nb56.log 2>&1 || fail "$step" $? $O/nb56.log
      cat $O/nb56.log ;;
    sprof:*)
      c=${step#sprof:}
      HNUMO_LIB=diag/libhnumo_diag.so timeout -k 10 300 python -u tools/stage_profile.py $c > $O/sprof_$c.txt 2>&1 || fail "$step" $? $O/sprof_$c.txt
      cat $O/sprof_$c.txt ;;
    bclprof:*)
      c=${step#bclprof:}
      HNUMO_LIB=diag/libhnumo_diag.so timeout -k 10 300 python -u tools/bcl_profile.py $c > $O/bclprof_$c.txt 2>&1 || fail "$step" $? $O/bclprof_$c.txt
      cat $O/bclprof_$c.txt ;;
    abbd:*)
      # abbd:<cfg[:stage]>:<KNOB>:<v1>/<v2>[/...]  tools/ab_breakdown.py (per-kernel step breakdown)
      IFS=: read -r _ cf md kn vs <<< "$step"
      [ "$md" = stage ] || { vs="$kn"; kn="$md"; md=""; }
      AB_REPS=${AB_REPS:-2} timeout -k 10 600 python -u tools/ab_breakdown.py $cf${md:+:$md} $kn ${vs//\// } >> $O/abbd.log 2>&1 || fail "$step" $? $O/abbd.log
      tail -4 $O/abbd.log ;;
    abbdl:*)
      # abbdl:<lib>:<cfg>  tools/ab_breakdown.py under HNUMO_LIB=<lib> (A/B of builds by the breakdown)
      x=${step#abbdl:}; lib=${x%%:*}; cf=${x#*:}
      [ "$lib" = default ] && lib=h-numo_amd/libhnumo_engine.so
      HNUMO_LIB=$lib AB_REPS=1 timeout -k 10 600 python -u tools/ab_breakdown.py $cf HNUMO_AB_LIB $(basename $lib) >> $O/abbd.log 2>&1 || fail "$step" $? $O/abbd.log
      tail -1 $O/abbd.log ;;
    abl:*)
      # abl:<lib>:<cfg>[,<cfg>...]  tools/ab_stage.py with HNUMO_LIB=<lib> (default: the product library)
      x=${step#abl:}; lib=${x%%:*}; cf=${x#*:}
      [ "$lib" = default ] && lib=h-numo_amd/libhnumo_engine.so
      HNUMO_LIB=$lib timeout -k 10 600 python -u tools/ab_stage.py ${cf//,/ } >> $O/abl.log 2>&1 || fail "$step" $? $O/abl.log
      tail -4 $O/abl.log ;;
    emu:*)
      # emu:W:R:cfg:order[:warmup:steps]  bench.py --emulate W:R under torch.distributed.run
      IFS=: read -r _ W R cf od wu ns <<< "$step"
      timeout -k 10 600 $TR bench.py --emulate $W:$R --config $cf --order $od --warmup ${wu:-3} --steps ${ns:-5} > $O/emu_${cf}_${od}.json 2> $O/emu_${cf}_${od}.err || fail "$step" $? $O/emu_${cf}_${od}.err
      cat $O/emu_${cf}_${od}.json ;;
    rank)
      timeout -k 10 600 python tools/c4_rank_cost.py > $O/c4_rank_cost.log 2>&1 || fail "$step" $? $O/c4_rank_cost.log
      tail -1 $O/c4_rank_cost.log ;;
    rankenv:*)
      # rankenv:<VAR>=<value>[,<VAR>=<value>]  tools/c4_rank_cost.py (rccl variant) under one environment setting
      kv=${step#rankenv:}
      env ${kv//,/ } timeout -k 10 600 python tools/c4_rank_cost.py --variants rccl --no-projection >> $O/rankenv.log 2>&1 || fail "$step" $? $O/rankenv.log
      echo "$kv: $(grep '"variant"' $O/rankenv.log | tail -1)" ;;
    rankprof)
      # kernel trace of the C4/8 rank (block vs self-neighbour RCCL) for the two-stream timeline
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/rankprof -o rp -- python tools/c4_rank_cost.py --variants block,rccl --steps 2 --no-projection > $O/rankprof.log 2>&1 || fail "$step" $? $O/rankprof.log
      tail -3 $O/rankprof.log ;;
    profiles)
      bash tools/gpu_profiles.sh $TAG || exit 1 ;;
    prof:*)
      bash tools/gpu_profiles.sh $TAG ${step#prof:} || exit 1 ;;
    ab:*)
      a=${step#ab:}
      timeout -k 10 900 python tools/ab_stage.py ${a//,/ } > $O/ab.log 2>&1 || fail "$step" $? $O/ab.log
      tail -20 $O/ab.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$(date +%T)] session $TAG done"
