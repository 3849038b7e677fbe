#!/bin/bash
# One GPU-box session: smoke, bench, GPU parity tests.  Every GPU step has its own time limit; a crash-like
# exit (abort, segfault, timeout, kill) ends the session immediately (no further GPU step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TESTS="${TESTS:-tests/test_gpu_parity.py}"
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"
  tail -5 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "crash-like exit, stopping"; exit $rc;; esac
  return 0
}
run smoke 400 python -c "import __graft_entry__ as g; g.smoke()"
run bench 600 python bench.py ${BENCH_ARGS:---steps 10 --warmup 2}
[ -n "$NO_TESTS" ] || run gpu_tests 1200 python -u -m pytest $TESTS -x -v -m gpu --timeout 400 --timeout-method thread
echo "=== done"
