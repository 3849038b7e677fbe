#!/bin/bash
# Same-box A/B of the config-2 step: this build vs an earlier one (LAB_LIB=tools/prev/lib_prev.so), alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2 3; do
  for v in cur prev; do
    if [ $v = prev ]; then export LAB_LIB=tools/prev/lib_prev.so; else unset LAB_LIB; fi
    timeout -k 10 120 python scripts/ab_lib.py --steps 30 --warmup 5 --no-cpu ${ARGS} > gpurun_out/ab_$v$i.log 2>&1 || { tail -5 gpurun_out/ab_$v$i.log; exit 1; }
    echo "$v $i $(grep 'ms/step' gpurun_out/ab_$v$i.log)"
  done
done
