#!/bin/bash
# GPU parity tests only ($TESTS, optional -k $K), one pytest process, per-test timeout; log under gpurun_out/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_gpu_configs.py tests/test_gpu_parity.py}"
timeout -k 10 ${TLIM:-1000} python -u -m pytest $TESTS -x -v -m gpu ${K:+-k "$K"} --timeout 400 --timeout-method thread \
  > gpurun_out/${LOG:-gpu_tests}.log 2>&1
rc=$?
tail -15 gpurun_out/${LOG:-gpu_tests}.log
exit $rc
