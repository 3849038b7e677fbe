#!/bin/bash
# Round 3: parity of the touched stage-4 / fan-out paths; config-4 / config-3 bench lines; the hot rank's per-step cost
# with the 21-bit split as 11 + 10 (default) and 10 + 11 (ORL_LB_CEIL=1).  Each GPU step has its own time limit; a
# crash-like or failing exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"; grep -E "ms/step|passed|failed|hottest|median" "gpurun_out/$name.log" | tail -4
  [ $rc = 0 ] || exit $rc
}
run chk_tests 600 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "lsd_offsets or config4 or config3 or stage4"
run chk_c4 180 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu
run chk_c3 300 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu
run chk_c3_old 300 env ORL_OFFSETS_SUFMIN=1 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu
run rank_cost 400 python scripts/rank_cost_lab.py 8 4 8
run rank_cost_ceil 400 env ORL_LB_CEIL=1 python scripts/rank_cost_lab.py 8 4 8
run chk_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof3 -o trace -- python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu
python3 scripts/kstats.py gpurun_out/c4prof3 | head -14
