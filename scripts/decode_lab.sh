#!/bin/bash
# f2 decode kernel lab: parity tests and leg-8 kernel times for the unstaged and LDS-staged variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/dlab}
mkdir -p $OUT
for v in ${MODES:-1}; do
  echo "=== ORL_DECODE_MODE=$v"
  ORL_DECODE_MODE=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k decode --timeout 240 --timeout-method thread > $OUT/tests_$v.log 2>&1
  rc=$?; tail -1 $OUT/tests_$v.log; [ $rc = 0 ] || exit $rc
  ORL_DECODE_MODE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$v -o trace -- python3 bench.py --config 8 --steps 5 --warmup 1 --no-cpu > $OUT/trace_$v.log 2>&1
  rc=$?; [ $rc = 0 ] || { tail -5 $OUT/trace_$v.log; exit $rc; }
  python3 -c "
import csv,glob
for f in glob.glob('$OUT/trace_$v/**/*kernel_stats.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'decode' in r['Name'] or 'k_route' in r['Name']: print(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3, 'us')
"
done
