#!/bin/bash
# Submit one gpurun step, retrying ONLY when gpurun reports that no slot/box was free (exit 3 or a "transient" status:
# nothing ran, nothing was charged).  Any run that actually executed ends the loop.  Usage: retry_gpu.sh <out-file> <cmd>
out=$1; shift
for i in $(seq 1 12); do
  timeout 1800 /usr/local/graft/bin/gpurun --timeout 1100 -- "$@" > "$out" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$out"; then sleep 120; continue; fi
  break
done
echo "FINISHED rc=$rc" >> "$out"
