# One gpurun job made of named steps, run in order; the first failing step ends the job
# (no GPU step runs after a crash, fault or time-out).  Replaces the one-off per-session
# wrappers of rounds 3-4 (tools/g_r3*.sh, tools/g_r4*.sh; in git history before round 5).
# usage: bash tools/gpu_job.sh TAG STEP [STEP ...]
#   tests[=PYTEST_ARGS]   pytest -m gpu over tests/ (or the given selection / -k args)
#   smoke                 __graft_entry__.smoke()
#   bench=WL[,ARGS]       bench.py --workload WL (driver defaults) -> gpurun_out/TAG_WL_bench.json
#   prof=WL               kernel trace + FETCH/WRITE passes of the driver command (tools/prof_bench.sh)
#   stall=WL              SQ stall / occupancy passes (tools/pmc_stall.sh)
#   valu=WL               SQ_INSTS_* pass (tools/pmc_valu.sh)
#   rows                  bench.py --rows (single drop-in calls) -> gpurun_out/TAG_rows.json
#   abenv=N,WL,ENV1,ENV2..  interleaved env A/B (tools/ab_envp.sh; ENV "K=V" or "-")
#   ablib=N,WL,TAG1,TAG2..  interleaved library-build A/B (tools/ab_lib.sh)
#   kprof=WL,TAG1,TAG2..    kernel-trace A/B of library builds (tools/kprof_lib.sh)
#   run=CMD               any command (spaces as '+'), e.g. run=python+tests/foo.py
# Args inside a step use ',' between fields and '+' for spaces.
set -o pipefail
TAG=${1:?tag}
shift
mkdir -p gpurun_out
for step in "$@"; do
  name=${step%%=*}
  arg=""
  [ "$step" != "$name" ] && arg=${step#*=}
  echo "== $TAG $step ($(date +%T))"
  case $name in
    tests)
      sel=${arg//+/ }
      timeout -k 10 1000 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu ${sel:-tests} \
        > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -30 gpurun_out/${TAG}_pytest.log; exit 1; }
      tail -3 gpurun_out/${TAG}_pytest.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      wl=${arg%%,*}
      extra=""
      [ "$arg" != "$wl" ] && extra=${arg#*,}
      extra=${extra//,/ }
      timeout -k 10 500 python bench.py --workload ${wl:-tum} ${extra//+/ } > gpurun_out/${TAG}_${wl:-tum}_bench.json \
        2> gpurun_out/${TAG}_${wl:-tum}_bench.err || { tail -20 gpurun_out/${TAG}_${wl:-tum}_bench.err; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_${wl:-tum}_bench.json').read().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('parity', {}).get('bit_exact'))" ;;
    prof)
      bash tools/prof_bench.sh $TAG ${arg:-tum} || exit 1 ;;
    stall)
      bash tools/pmc_stall.sh ${TAG}_${arg:-tum} ${arg:-tum} || exit 1 ;;
    valu)
      bash tools/pmc_valu.sh $TAG ${arg:-tum} || exit 1 ;;
    rows)
      timeout -k 10 600 python bench.py --rows > gpurun_out/${TAG}_rows.json 2> gpurun_out/${TAG}_rows.err \
        || { tail -20 gpurun_out/${TAG}_rows.err; exit 1; } ;;
    abenv)
      IFS=',' read -r -a a <<< "$arg"
      envs=()
      for e in "${a[@]:2}"; do envs+=("${e//+/ }"); done
      bash tools/ab_envp.sh ${a[0]} ${a[1]} "${envs[@]}" || exit 1 ;;
    ablib)
      IFS=',' read -r -a a <<< "$arg"
      bash tools/ab_lib.sh ${a[0]} ${a[1]} "${a[@]:2}" || exit 1 ;;
    kprof)
      IFS=',' read -r -a a <<< "$arg"
      bash tools/kprof_lib.sh ${a[0]} "${a[@]:1}" || exit 1 ;;
    run)
      timeout -k 10 900 ${arg//+/ } || exit 1 ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== $TAG done"
