#!/bin/bash
# A GPU-box session: optional GPU tests ($TESTS, -k $K), then bench legs ($LEGS: "name:[VAR=v ...] args;name:args").  Every GPU step has
# its own time limit; a crash-like exit (abort, segfault, timeout, kill) ends the session (no further GPU step).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name exit $rc"
  tail -4 "gpurun_out/$name.log"
  case $rc in 124|134|137|139) echo "crash-like exit, stopping"; exit $rc;; esac
  return 0
}
if [ -n "$TESTS" ]; then
  step tests ${TLIM:-900} python -u -m pytest $TESTS -x -v -m gpu ${K:+-k "$K"} --timeout 400 --timeout-method thread
fi
IFS=';' read -ra LG <<< "$LEGS"
for leg in "${LG[@]}"; do
  [ -z "$leg" ] && continue
  name=${leg%%:*}; a=${leg#*:}
  envs=(); args=()
  for tok in $a; do  # leading VAR=value tokens set the leg's environment (e.g. ORL_SCAN3=1)
    if [ ${#args[@]} -eq 0 ] && [[ $tok == [A-Z]*=* ]]; then envs+=("$tok"); else args+=("$tok"); fi
  done
  step "bench_$name" ${BLIM:-400} env "${envs[@]}" python bench.py "${args[@]}"
  grep '^{' "gpurun_out/bench_$name.log" > "gpurun_out/bench_$name.json" || true
done
echo "=== done"
