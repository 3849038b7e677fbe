#!/bin/bash
# Round-3 final evidence, part A: k_part_lb load-group A/B, the full GPU suite, the default bench line and bench lines
# of configs 1, 3, 4, 5 with their CPU baselines.  Each GPU step has its own time limit; a failing or crash-like exit
# of a test step stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03f
for v in g1 main g4; do
  if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=tools/$v/lib.so; fi
  timeout -k 10 300 python scripts/rank_cost_lab.py 8 4 8 > gpurun_out/r03f/part_$v.log 2>&1 || { tail -5 gpurun_out/r03f/part_$v.log; exit 1; }
  echo "$v: $(grep 'hop 1' gpurun_out/r03f/part_$v.log)"
done
unset LAB_LIB
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/r03f/gpu_tests.log 2>&1
rc=$?; echo "gpu tests exit $rc: $(tail -1 gpurun_out/r03f/gpu_tests.log)"; [ $rc = 0 ] || { tail -30 gpurun_out/r03f/gpu_tests.log; exit $rc; }
timeout -k 10 120 python bench.py --steps 20 --warmup 5 > gpurun_out/r03f/c2.json 2> gpurun_out/r03f/c2.log
rc=$?; echo "default bench exit $rc: $(grep 'rank 0' gpurun_out/r03f/c2.log)"; case $rc in 0) ;; *) exit $rc;; esac
for c in 1 3 4 5; do
  timeout -k 10 400 python bench.py --config $c --steps 10 --warmup 2 > gpurun_out/r03f/c$c.json 2> gpurun_out/r03f/c$c.log
  rc=$?; echo "config $c exit $rc: $(grep -E 'rank 0:|config [1345]' gpurun_out/r03f/c$c.log | tail -1)"
  case $rc in 0) ;; *) tail -5 gpurun_out/r03f/c$c.log; exit $rc;; esac
done
echo "=== done"
