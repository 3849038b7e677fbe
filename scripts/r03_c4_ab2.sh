#!/bin/bash
# Round 3: config-4 grid A/B (ORL_ROUTE_MIN_WG: route tiles per launch) x fan-out messages per thread (ORL_FAN_U), then a
# kernel trace of the default; each GPU step under its own time limit, a crash-like exit stops the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
run() {  # name limit cmd...
  local name=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  [ $rc = 0 ] || { echo "=== $name exit $rc"; tail -5 "gpurun_out/$name.log"; exit $rc; }
}
for v in ${VARIANTS:-"ORL_FAN_U=1" "ORL_ROUTE_MIN_WG=4096" "ORL_ROUTE_MIN_WG=8192" "ORL_ROUTE_MIN_WG=4096 ORL_FAN_U=2" "ORL_ROUTE_MIN_WG=16384" "ORL_FAN_U=1"}; do
  tag=$(echo $v | tr ' =' '__')
  run "c4_$tag" 180 env $v python bench.py --config ${CFG:-4} --steps 30 --warmup 5 --no-cpu
  grep '^{' "gpurun_out/c4_$tag.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); p=d.get('pipeline',{}); print('$v', round(d['ms_per_step'],4), p)"
done
run c4_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c4prof -o trace -- python3 bench.py --config ${CFG:-4} --steps 10 --warmup 2 --no-cpu
python3 scripts/kstats.py gpurun_out/c4prof | head -30
