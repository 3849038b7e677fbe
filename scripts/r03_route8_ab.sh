#!/bin/bash
# k_route8_multi (the 8-B owner route with U records per thread and step): node + narrow-record parity with U = 2 and 4,
# then the hot/median rank's route (rank_cost_lab) and the 8-rank rehearsal for U = 1, 2, 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r8
for u in 2 4; do
  ORL_ROUTE8_U=$u timeout -k 10 700 python -u -m pytest tests/test_gpu_node.py tests/test_gpu_parity.py -x -q -m gpu --timeout 500 \
    --timeout-method thread -k "node or narrow" > gpurun_out/r8/tests_u$u.log 2>&1
  rc=$?; echo "tests U=$u exit $rc: $(tail -1 gpurun_out/r8/tests_u$u.log)"; [ $rc = 0 ] || { tail -30 gpurun_out/r8/tests_u$u.log; exit $rc; }
done
for u in 1 2 4 2 1; do
  ORL_ROUTE8_U=$u timeout -k 10 300 python scripts/rank_cost_lab.py 8 4 8 > gpurun_out/r8/rank_u$u.log 2>&1 || exit 1
  echo "U=$u: $(grep hottest gpurun_out/r8/rank_u$u.log | cut -c1-95) | $(grep median gpurun_out/r8/rank_u$u.log | cut -c1-95)"
done
for u in 1 2 1 2; do
  ORL_ROUTE8_U=$u timeout -k 10 300 python bench.py --local-ranks 8 --config 3 --steps 5 --warmup 2 > gpurun_out/r8/reh_u$u.log 2>&1 || exit 1
  echo "U=$u: $(grep rehearsal gpurun_out/r8/reh_u$u.log | cut -c1-70)"
done
