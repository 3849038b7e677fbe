#!/bin/bash
# k_part_lb<8> header load groups per tile: 1 (round 2), 2 (default build), 4 -- the hop-1 partition of one rank's 32M
# messages in 4 calls (rank_cost_lab.py), alternating builds; then the node GPU tests on the default build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for i in 1 2; do
  for v in g1 main g4; do
    if [ $v = main ]; then unset LAB_LIB; else export LAB_LIB=tools/$v/lib.so; fi
    timeout -k 10 400 python scripts/rank_cost_lab.py 8 4 8 > gpurun_out/part_$v$i.log 2>&1 || { tail -5 gpurun_out/part_$v$i.log; exit 1; }
    echo "$v $i: $(grep 'hop 1' gpurun_out/part_$v$i.log) | $(grep hottest gpurun_out/part_$v$i.log | cut -c1-90)"
  done
done
unset LAB_LIB
timeout -k 10 900 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_parity.py -x -q -m gpu --timeout 600 --timeout-method thread -k "node or partition or wire" > gpurun_out/part_tests.log 2>&1; rc=$?
tail -3 gpurun_out/part_tests.log; exit $rc
