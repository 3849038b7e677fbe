#!/bin/bash
# Run GPU commands in order, one per line of $CMDS ("name|seconds|command"), each under its own time limit, output to
# $OUT/<name>.log.  Exit status 0 or 1 (a failed check or test) continues; anything else (abort, fault, time limit) stops.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/cmds}
mkdir -p $OUT
while IFS='|' read -r name secs cmd; do
  [ -z "$name" ] && continue
  timeout -k 10 $secs bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  echo "== $name exit $rc"; grep -vE "amdgpu.ids|^\s*$" $OUT/$name.log | tail -${TAIL:-6}
  case $rc in 0|1) ;; *) echo "stopping after $name"; exit $rc;; esac
done <<< "$CMDS"
