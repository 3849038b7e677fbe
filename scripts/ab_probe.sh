#!/bin/bash
# GPU parity tests, then bench config 2 with the 8-B / 16-B compact probe table and the 32-B table (ORL_NO_PROBE8/16).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
[ $rc = 0 ] || { tail -60 gpurun_out/gpu_tests.log; exit $rc; }
for v in 0 1 8 0 1 8; do
  ORL_NO_PROBE8=$([ $v = 8 ] && echo 1 || echo 0) ORL_NO_PROBE16=$([ $v = 1 ] && echo 1 || echo 0) timeout -k 10 300 python bench.py --steps 10 --warmup 2 --no-cpu ${BENCH_ARGS} > gpurun_out/ab_$v.log 2>&1
  rc=$?; echo "variant $v (0: 8-B probe table if it fits, 8: 16-B, 1: 32-B) exit $rc"; grep "rank 0:" gpurun_out/ab_$v.log
  case $rc in 0) ;; *) tail -20 gpurun_out/ab_$v.log; exit $rc;; esac
done
