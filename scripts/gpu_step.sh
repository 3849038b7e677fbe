#!/bin/bash
# One parameterised GPU session step (replaces the per-experiment r03_*.sh wrappers).  Every step has its own time limit;
# a failing, aborted, faulted or timed-out step ends the script (nothing else runs on the GPU after it).
#   OUT=gpurun_out/<name>      output directory
#   TESTS="<pytest targets>"   GPU tests to run first (K=<-k expr> optional); empty: none
#   AB="NAME=v1,v2;..."        bench A/B: one default-config bench line per value of each env var (BENCH_ARGS applies)
#   BENCH_ARGS="..."           bench arguments (default --steps 20 --warmup 5 --no-cpu)
#   CONFIGS="1 3 4 5"          extra bench lines, one per config (--config c --steps 10 --warmup 2)
#   PROF=1                     rocprofv3 kernel trace of the default bench (PROF_ARGS; stats to $OUT/trace)
#   PMC="g1;g2"                extra rocprofv3 --pmc passes (one per ';'-separated group) over PROF_ARGS (PMC_ARGS: extra
#                              rocprofv3 options, e.g. --kernel-include-regex k_probe_slice)
#   LAB="cmd"                  an extra command (e.g. python scripts/rank_cost_lab.py 8 4 8), 300 s limit
#   LAB_ENVS="A=1;A=2"         run LAB once per environment (lab_<i>.log)
#   LAB2="cmd" LAB2_ENV="N=v"  a second lab command with its environment
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/step}
mkdir -p $OUT
BENCH_ARGS=${BENCH_ARGS:---steps 20 --warmup 5 --no-cpu}
PROF_ARGS=${PROF_ARGS:---steps 5 --warmup 1 --no-cpu}
stop() { case $1 in 0) ;; *) echo "step exit $1: stopping"; exit $1;; esac; }

if [ -n "$TESTS" ]; then
  timeout -k 10 ${TLIM:-900} python -u -m pytest $TESTS -x -v -m gpu ${K:+-k "$K"} --timeout 400 --timeout-method thread --capture=tee-sys \
    > $OUT/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests exit $rc: $(tail -1 $OUT/gpu_tests.log)"
  [ $rc = 0 ] || { grep -E "FAILED|Error|error" $OUT/gpu_tests.log | head -20; tail -25 $OUT/gpu_tests.log; exit $rc; }
fi
if [ -n "$AB" ]; then
  IFS=';' read -ra VARS <<< "$AB"
  for spec in "${VARS[@]}"; do
    name=${spec%%=*}; vals=${spec#*=}
    IFS=',' read -ra VS <<< "$vals"
    for rep in 1 2; do
      for v in "${VS[@]}"; do
        f=$OUT/ab_${name}_${v//\//_}_$rep
        env $name=$v timeout -k 10 180 python bench.py $BENCH_ARGS > $f.json 2> $f.log
        rc=$?; echo "$name=$v rep $rep: $(python3 -c "import json,sys; d=json.load(open('$f.json')); print(d['ms_per_step'], 'ms', d.get('roofline',{}).get('frac'))" 2>/dev/null)"
        stop $rc
      done
    done
  done
fi
if [ -n "$CONFIGS" ]; then
  for c in $CONFIGS; do
    timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 ${CFG_ARGS} > $OUT/c$c.json 2> $OUT/c$c.log
    rc=$?; echo "config $c exit $rc: $(python3 -c "import json; d=json.load(open('$OUT/c$c.json')); print(d['ms_per_step'], 'ms', d['value'], d['unit'])" 2>/dev/null)"
    stop $rc
  done
fi
if [ "${PROF:-0}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 bench.py $PROF_ARGS > $OUT/trace.log 2>&1
  rc=$?; echo "trace exit $rc"; stop $rc
  python3 scripts/kstats.py $OUT/trace > $OUT/kernel_stats.txt 2>&1 && head -25 $OUT/kernel_stats.txt
fi
if [ -n "$PMC" ]; then
  IFS=';' read -ra GRPS <<< "$PMC"
  i=0
  for grp in "${GRPS[@]}"; do
    i=$((i+1))
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $grp $PMC_ARGS --output-format csv -d $OUT/pmc$i -o pmc -- python3 bench.py $PROF_ARGS > $OUT/pmc$i.log 2>&1
    rc=$?; echo "pmc$i ($grp) exit $rc"; stop $rc
  done
  python3 scripts/pmc_summary.py $OUT > $OUT/pmc_summary.txt 2>&1; head -40 $OUT/pmc_summary.txt
fi
if [ -n "$LAB" ] && [ -n "$LAB_ENVS" ]; then  # LAB once per ';'-separated environment (e.g. "LAB_LIB=a.so;LAB_LIB=b.so")
  IFS=';' read -ra LES <<< "$LAB_ENVS"
  i=0
  for le in "${LES[@]}"; do
    i=$((i+1))
    env ${le:-_LAB=1} timeout -k 10 300 $LAB > $OUT/lab_$i.log 2>&1
    rc=$?; echo "lab $i ($le) exit $rc"; grep -v amdgpu.ids $OUT/lab_$i.log | tail -6; stop $rc
  done
elif [ -n "$LAB" ]; then
  timeout -k 10 300 $LAB > $OUT/lab.log 2>&1
  rc=$?; echo "lab exit $rc"; tail -15 $OUT/lab.log; stop $rc
fi
if [ -n "$LAB2" ]; then  # a second lab command (LAB2_ENV="NAME=value": its environment)
  env ${LAB2_ENV:-_LAB2=1} timeout -k 10 300 $LAB2 > $OUT/lab2.log 2>&1
  rc=$?; echo "lab2 exit $rc"; tail -15 $OUT/lab2.log; stop $rc
fi
echo "=== done"
