#!/bin/bash
# Round-3 measurements, part A: per-rank cost at 8 ranks (hot-key path on / off), the 8-rank rehearsal, config 4 / 5 /
# narrow host-io bench lines.  Every GPU step has its own time limit; a crash-like exit ends the session.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r03m
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/r03m/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"; tail -3 "gpurun_out/r03m/$name.log"
  case $rc in 124|134|137|139) echo "crash-like exit, stopping"; exit $rc;; esac
  return 0
}
step rank_cost_hot 300 python -u scripts/rank_cost_lab.py 8 4 8
step rank_cost_nohot 300 env ORL_NO_HOT=1 python -u scripts/rank_cost_lab.py 8 4 8
step rehearsal8_c3 300 python -u bench.py --local-ranks 8 --config 3 --steps 5 --warmup 2
step c4 300 python -u bench.py --config 4 --steps 10 --warmup 2
step c5 300 python -u bench.py --config 5 --steps 20 --warmup 2
step hostio_narrow 300 python -u bench.py --host-io narrow --steps 5 --warmup 1 --no-cpu
step hostio_pinned 300 python -u bench.py --host-io pinned --steps 5 --warmup 1 --no-cpu
for f in gpurun_out/r03m/*.log; do grep -h '^{' "$f" > "${f%.log}.json" 2>/dev/null || true; done
echo "=== done"
