#!/bin/bash
# Round-3 final evidence, part B: rocprofv3 kernel trace + PMC passes of config 2 and config 4, the per-rank cost at 8
# ranks and the 8-rank one-GPU rehearsal of config 3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r03g
OUT=gpurun_out/r03g/c2 bash scripts/profile.sh || exit $?
OUT=gpurun_out/r03g/c4 BENCH_ARGS="--config 4 --steps 3 --warmup 1 --no-cpu" PMC_GROUPS="FETCH_SIZE;TCC_HIT_sum TCC_MISS_sum;WRITE_SIZE" \
  bash scripts/profile.sh || exit $?
timeout -k 10 300 python -u scripts/rank_cost_lab.py 8 4 8 > gpurun_out/r03g/rank_cost.log 2>&1; echo "rank cost exit $?"
LAB_LIB=tools/g4w6/lib.so timeout -k 10 300 python -u scripts/rank_cost_lab.py 8 4 8 > gpurun_out/r03g/rank_cost_g4w6.log 2>&1; echo "g4w6: $(grep "hop 1" gpurun_out/r03g/rank_cost_g4w6.log)"
grep -E "hop 1|hottest|median" gpurun_out/r03g/rank_cost.log
timeout -k 10 300 python -u bench.py --local-ranks 8 --config 3 --steps 5 --warmup 2 > gpurun_out/r03g/rehearsal8_c3.json 2> gpurun_out/r03g/rehearsal8_c3.log
echo "rehearsal exit $?"; tail -2 gpurun_out/r03g/rehearsal8_c3.log
echo "=== done"
