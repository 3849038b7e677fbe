#!/bin/bash
# Hop 2's remote-flag round (the owner's route sets a flag; the count pass only when some rank forwards): node parity,
# then the 8-rank one-GPU rehearsal of config 3 against the previous build, alternating.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/rf
timeout -k 10 900 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_configs.py -x -q -m gpu --timeout 600 --timeout-method thread \
  -k "node or fanout_expand" > gpurun_out/rf/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 gpurun_out/rf/tests.log)"; [ $rc = 0 ] || { tail -30 gpurun_out/rf/tests.log; exit $rc; }
for i in 1 2; do
  for v in cur prev; do
    if [ $v = prev ]; then export LAB_LIB=tools/prev/lib_prev.so; else unset LAB_LIB; fi
    timeout -k 10 300 python scripts/ab_lib.py --local-ranks 8 --config 3 --steps 5 --warmup 2 > gpurun_out/rf/reh_$v$i.log 2>&1 || { tail -5 gpurun_out/rf/reh_$v$i.log; exit 1; }
    echo "$v $i: $(grep 'rehearsal' gpurun_out/rf/reh_$v$i.log | cut -c1-80)"
  done
done
