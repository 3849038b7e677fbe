#!/bin/bash
# u16 histogram count rows: parity of every stage-4 path, then same-box A/B against the previous build (config 2, config 4,
# hot rank at 8 ranks).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/u16
timeout -k 10 900 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py tests/test_gpu_node.py -x -q -m gpu --timeout 600 \
  --timeout-method thread > gpurun_out/u16/tests.log 2>&1
rc=$?; echo "tests exit $rc: $(tail -1 gpurun_out/u16/tests.log)"; [ $rc = 0 ] || { tail -30 gpurun_out/u16/tests.log; exit $rc; }
for i in 1 2; do
  for v in cur prev; do
    if [ $v = prev ]; then export LAB_LIB=tools/prev/lib_prev.so; else unset LAB_LIB; fi
    timeout -k 10 120 python scripts/ab_lib.py --steps 30 --warmup 5 --no-cpu > gpurun_out/u16/c2_$v$i.log 2>&1 || exit 1
    timeout -k 10 120 python scripts/ab_lib.py --config 4 --steps 30 --warmup 5 --no-cpu > gpurun_out/u16/c4_$v$i.log 2>&1 || exit 1
    echo "$v $i c2: $(grep 'ms/step' gpurun_out/u16/c2_$v$i.log | cut -c1-110) | c4: $(grep 'ms/step' gpurun_out/u16/c4_$v$i.log | cut -c1-100)"
  done
done
for v in cur prev; do
  if [ $v = prev ]; then export LAB_LIB=tools/prev/lib_prev.so; else unset LAB_LIB; fi
  timeout -k 10 300 python scripts/rank_cost_lab.py 8 4 8 > gpurun_out/u16/rank_$v.log 2>&1 || exit 1
  echo "$v: $(grep hottest gpurun_out/u16/rank_$v.log | cut -c1-100) | $(grep median gpurun_out/u16/rank_$v.log | cut -c1-100)"
done
