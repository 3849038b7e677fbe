#!/bin/bash
# Round-3 measurements, part B: rocprofv3 kernel trace + PMC passes of config 2 (the headline) and config 4, and the
# config-3 one-GPU bench line.  Each rocprofv3 run has its own time limit; PMC passes run alone (no tracing domains).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03p
OUT=gpurun_out/r03p/c2 bash scripts/profile.sh || exit $?
OUT=gpurun_out/r03p/c4 BENCH_ARGS="--config 4 --steps 3 --warmup 1 --no-cpu" PMC_GROUPS="FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum;WRITE_SIZE" \
  bash scripts/profile.sh || exit $?
timeout -k 10 400 python -u bench.py --config 3 --steps 5 --warmup 2 > gpurun_out/r03p/c3_1gpu.json 2> gpurun_out/r03p/c3_1gpu.log
echo "c3 exit $?"; tail -2 gpurun_out/r03p/c3_1gpu.log
echo "=== done"
