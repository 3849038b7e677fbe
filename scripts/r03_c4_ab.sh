#!/bin/bash
# Round 3: config-4 A/B (fan-out route messages per thread ORL_FAN_U, LSD offsets form ORL_OFFSETS_SUFMIN) after the
# parity tests of the touched paths; every GPU step under its own time limit, a crash-like exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"; tail -3 "gpurun_out/$name.log"
  [ $rc = 0 ] || exit $rc
}
run c4_tests 600 python -u -m pytest tests/test_gpu_configs.py -x -v -m gpu --timeout 300 --timeout-method thread \
  -k "lsd_offsets or config4 or config5 or fanout or stage4 or config3"
for v in "ORL_FAN_U=1" "ORL_FAN_U=2" "ORL_FAN_U=4" "ORL_FAN_U=1 ORL_OFFSETS_SUFMIN=1" "ORL_FAN_U=2"; do
  tag=$(echo $v | tr ' =' '__')
  run "c4_$tag" 180 env $v python bench.py --config 4 --steps 30 --warmup 5 --no-cpu
  grep '^{' "gpurun_out/c4_$tag.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', d['ms_per_step'], d.get('roofline',{}).get('achieved'), d.get('stages_ms', ''))"
done
