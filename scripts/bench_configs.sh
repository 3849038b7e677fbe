#!/bin/bash
# GPU parity tests, then bench.py over the SURVEY §8(d) workloads (configs 2-5), one JSON line each.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/configs
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 400 --timeout-method thread > gpurun_out/configs/gpu_tests.log 2>&1
  rc=$?; echo "gpu tests exit $rc: $(tail -1 gpurun_out/configs/gpu_tests.log)"
  case $rc in 0) ;; *) tail -30 gpurun_out/configs/gpu_tests.log; exit $rc;; esac
fi
for c in ${CONFIGS:-2 3 4 5}; do
  timeout -k 10 500 python bench.py --config $c --steps ${STEPS:-10} --warmup 2 ${BENCH_EXTRA:-} > gpurun_out/configs/c$c.json 2> gpurun_out/configs/c$c.log
  rc=$?; echo "config $c exit $rc: $(grep -E 'rank 0:|config [45]:' gpurun_out/configs/c$c.log | tail -1)"
  case $rc in 0) ;; 124|134|137|139) tail -5 gpurun_out/configs/c$c.log; exit $rc;; *) tail -5 gpurun_out/configs/c$c.log;; esac
done
