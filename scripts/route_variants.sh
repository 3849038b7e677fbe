#!/bin/bash
# A/B kernel structure variants (ORL_ROUTE_VARIANT / ORL_RADIX_VARIANT) on the config-2 bench; parity-check candidates.
# VARIANTS="r:x ..." pairs of route:radix variant numbers; TEST_VARIANTS likewise.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/var
for v in ${VARIANTS:-0:0}; do
  r=${v%%:*}; x=${v##*:}
  ORL_ROUTE_VARIANT=$r ORL_RADIX_VARIANT=$x timeout -k 10 240 python bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/var/v$r-$x.json 2> gpurun_out/var/v$r-$x.log
  rc=$?; echo "variant $v exit $rc: $(grep 'rank 0:' gpurun_out/var/v$r-$x.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
for v in ${TEST_VARIANTS:-}; do
  r=${v%%:*}; x=${v##*:}
  ORL_ROUTE_VARIANT=$r ORL_RADIX_VARIANT=$x timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/var/test_v$r-$x.log 2>&1
  rc=$?; echo "tests variant $v exit $rc: $(tail -1 gpurun_out/var/test_v$r-$x.log)"
  case $rc in 124|134|137|139) exit $rc;; esac
done
