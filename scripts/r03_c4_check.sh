#!/bin/bash
# Round 3: parity of the stage-4 / fan-out paths, then config-4 and config-3 (one GPU) bench lines with a kernel trace.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"; tail -2 "gpurun_out/$name.log"
  [ $rc = 0 ] || exit $rc
}
run chk_tests 600 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_parity.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "${K:-lsd_offsets or config4 or config5 or fanout or stage4 or config3 or chirper or random_batches}"
run chk_c4 180 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu
run chk_c4_old 180 env ORL_FAN_MIN_WG=2048 ORL_OFFSETS_SUFMIN=1 python bench.py --config 4 --steps 30 --warmup 5 --no-cpu
run chk_c3 300 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu
run chk_c3_old 300 env ORL_OFFSETS_SUFMIN=1 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu
run chk_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof2 -o trace -- python3 bench.py --config 4 --steps 10 --warmup 2 --no-cpu
python3 scripts/kstats.py gpurun_out/c4prof2 | head -16
