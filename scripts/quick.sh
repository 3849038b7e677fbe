#!/bin/bash
# Quick GPU iteration: parity tests (optionally filtered by $K), then a kernel-trace profile of bench.py.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu ${K:+-k "$K"} --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
rc=$?; tail -3 gpurun_out/gpu_tests.log
[ $rc = 0 ] || { tail -40 gpurun_out/gpu_tests.log; exit $rc; }
PMC=0 OUT=${OUT:-gpurun_out/profq} BENCH_ARGS="${BENCH_ARGS:---steps 5 --warmup 1 --no-cpu}" bash scripts/profile.sh
