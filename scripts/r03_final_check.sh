#!/bin/bash
# End-of-session check of the committed build: the full GPU suite, smoke(), the default bench line, config 4.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03h
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 400 --timeout-method thread > gpurun_out/r03h/gpu_tests.log 2>&1
rc=$?; echo "gpu tests exit $rc: $(tail -1 gpurun_out/r03h/gpu_tests.log)"; [ $rc = 0 ] || { tail -30 gpurun_out/r03h/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r03h/smoke.log 2>&1
rc=$?; echo "smoke exit $rc: $(tail -1 gpurun_out/r03h/smoke.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 120 python bench.py > gpurun_out/r03h/default.json 2> gpurun_out/r03h/default.log
rc=$?; echo "default bench exit $rc: $(grep 'rank 0:' gpurun_out/r03h/default.log)"; [ $rc = 0 ] || exit $rc
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 2 > gpurun_out/r03h/c4.json 2> gpurun_out/r03h/c4.log
echo "config 4 exit $?: $(grep 'config 4:' gpurun_out/r03h/c4.log)"
